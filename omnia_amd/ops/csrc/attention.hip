// Paged attention for the in-node engine on gfx950.
//
// KV cache layout (shared with rope_kv in elementwise.hip):
//     k_cache, v_cache : [num_blocks, Hkv, BS, 128] bf16
// i.e. one kv-head's rows of a page are contiguous, so a 16-lane group reads a
// whole 256-B token row and a wave-instruction reads 4 consecutive tokens = 1 KiB.
//
// decode  : split-K ("flash-decoding") over partitions of the context, GQA
//           group of G query heads per workgroup sharing one K/V stream;
//           Q.K^T on the MFMA (16x16x32 bf16, heads padded to 16 columns),
//           softmax in LDS, P.V on the VALU (8 dims per lane), partitions merged
//           by a second tiny kernel.
// prefill : flash-attention over (cached prefix + new tokens) with causal
//           offset, 64 query rows x 1 head per workgroup (16 rows per wave),
//           K/V tiles of 64 keys gathered from pages into XOR-swizzled LDS,
//           S^T = K.Q^T so each lane owns one query row (softmax row stats are
//           lane-local + 2 shuffles), P^T reused in-register as the B operand of
//           O^T = V^T.P^T with V^T fragments from ds_read_b64_tr_b16.
#include <stdlib.h>

#include "common.h"

using namespace omnia;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float4v mfma16(short8 a, short8 b, float4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

constexpr int D = 128;

// ============================================================== decode
// Length-balanced split (split_t > 0): a sequence of `len` keys is cut into
// ns = clamp(ceil(len / split_min), ceil(len / cap), split_t) partitions of equal
// page-aligned length -- decided on the device from the live length, so a graph
// captured once splits every context evenly (a host-chosen fixed partition
// leaves one workgroup per (sequence, kv head) at short contexts when the batch
// has few such pairs, e.g. one Llama-3-70B TP=8 rank).  cap (the LDS score
// tile) and BS divide each other's multiples: pl <= cap always.
__device__ __forceinline__ int decode_part_len(int len, int cap, int split_t, int split_min,
                                               int bs) {
  if (split_t <= 0) return cap;
  int ns = min(split_t, (len + split_min - 1) / split_min);
  ns = max(ns, max((len + cap - 1) / cap, 1));
  const int pl = ((len + ns - 1) / ns + bs - 1) / bs * bs;
  return min(pl, cap);
}

// grid: (B, Hkv, max_parts)   block: 64 * NW (NW = 2 or 4 waves)
// UG: 16-key groups whose K loads one wave issues before its first MFMA (and,
// for UG > 1, the first V batch is issued ahead of the softmax) -- the memory-
// level parallelism of one workgroup, which at short contexts (one workgroup
// streams a whole ~600-token context) sets the kernel's speed, not HBM.
// U: V rows (16 B per lane each) one wave keeps in flight under the P.V of the
// previous batch -- the same parallelism for phase 3.
template <int G, int BS, int UG, int NW, int U>
__global__ __launch_bounds__(64 * NW) void decode_attn_kernel(
    bf16_t* __restrict__ out, float* __restrict__ part_o, float* __restrict__ part_ml,
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ seq_lens,
    int hkv, int64_t q_stride, int part_size, int max_parts, float scale_log2, int split_t,
    int split_min) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* stat = reinterpret_cast<float*>(smem);                    // [2*G] (padded to 16 floats)
  float* scores = stat + 16;                                       // [G][part_size]
  // [NW][G][D] wave partials of P.V: aliases `scores` (written after every wave's
  // last scores read), so a workgroup holds one [G][part_size] score tile
  float* red = scores;
  int* pages = reinterpret_cast<int*>(scores + (G * part_size > NW * G * D ? G * part_size
                                                                            : NW * G * D));

  const int b = blockIdx.x, kvh = blockIdx.y, part = blockIdx.z;
  const int len = seq_lens[b];
  if (len <= 0) return;
  const int pl = decode_part_len(len, part_size, split_t, split_min, BS);
  const int p0 = part * pl;
  if (p0 >= len) return;
  const int n = min(pl, len - p0);
  const int nparts = (len + pl - 1) / pl;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int h0 = kvh * G;

  for (int i = tid; i < (n + BS - 1) / BS; i += 64 * NW)
    pages[i] = block_tables[(int64_t)b * bt_stride + p0 / BS + i];

  // Q^T as the MFMA B operand: column = head (l&15, only < G real), k = dims
  short8 qf[4];
  {
    const int g = lane & 15;
    const int hh = h0 + (g < G ? g : 0);
    const bf16_t* qrow = q + (int64_t)b * q_stride + hh * D;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      short8 v = *reinterpret_cast<const short8*>(qrow + kk * 32 + 8 * (lane >> 4));
      if (g >= G) v = short8{0, 0, 0, 0, 0, 0, 0, 0};
      qf[kk] = v;
    }
  }
  __syncthreads();

  // ---- phase 1: scores. each wave takes 16-key groups round-robin, UG per
  // pass with all their K loads in flight before the first MFMA (groups past
  // the end re-read the last key: branch-free, hits in cache).
  const int ngroups = (n + 15) / 16;
  for (int grp0 = w; grp0 < ngroups; grp0 += NW * UG) {
    short8 a[UG][4];
#pragma unroll
    for (int u = 0; u < UG; ++u) {
      const int key = (grp0 + NW * u) * 16 + (lane & 15);  // this lane's A-row key
      const int kk_ = min(key, n - 1);
      const int tok = p0 + kk_;
      const bf16_t* krow = kc + (((int64_t)pages[kk_ / BS] * hkv + kvh) * BS + (tok % BS)) * D;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
        a[u][kk] = *reinterpret_cast<const short8*>(krow + kk * 32 + 8 * (lane >> 4));
    }
#pragma unroll
    for (int u = 0; u < UG; ++u) {
      const int grp = grp0 + NW * u;
      if (grp >= ngroups) break;
      float4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) acc = mfma16(a[u][kk], qf[kk], acc);
      // acc[r] = S^T[key grp*16 + 4*(lane>>4) + r][head lane&15]
      const int g = lane & 15;
      if (g < G) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int kidx = grp * 16 + 4 * (lane >> 4) + r;
          if (kidx < n) scores[g * part_size + kidx] = acc[r] * scale_log2;
        }
      }
    }
  }
  // first V batch of phase 3 in flight across the softmax (plain loads survive
  // the barriers); lane = (token sub-index tg = lane>>4, dim chunk ch = lane&15)
  const int tg = lane >> 4, ch = lane & 15;
  short8 vv[U];
  auto vload = [&](int base) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = min(base + u * 4 * NW + tg, n - 1);
      const int tok = p0 + t;
      vv[u] = *reinterpret_cast<const short8*>(
          vc + (((int64_t)pages[t / BS] * hkv + kvh) * BS + (tok % BS)) * D + ch * 8);
    }
  };
  if (UG > 1) vload(w * 4);
  __syncthreads();

  // ---- phase 2: softmax per head (wave w handles heads w, w+NW, ...)
  for (int g = w; g < G; g += NW) {
    float m = -INFINITY;
    for (int i = lane; i < n; i += 64) m = fmaxf(m, scores[g * part_size + i]);
    m = wave_max(m);
    float s = 0.f;
    for (int i = lane; i < n; i += 64) {
      const float p = exp2f(scores[g * part_size + i] - m);
      scores[g * part_size + i] = p;
      s += p;
    }
    s = wave_sum(s);
    if (lane == 0) {
      stat[2 * g] = m;
      stat[2 * g + 1] = s;
    }
  }
  __syncthreads();

  // ---- phase 3: P.V. lane = (token sub-index tg = lane>>4, dim chunk ch = lane&15)
  float acc[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[g][j] = 0.f;
  for (int base = w * 4; base < n; base += 4 * NW * U) {
    if (UG == 1) vload(base);
    short8 cur[U];
#pragma unroll
    for (int u = 0; u < U; ++u) cur[u] = vv[u];
    if (UG > 1) vload(base + 4 * NW * U);  // next batch (clamped past the end)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ti = base + u * 4 * NW + tg;
      if (ti < n) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const float p = scores[g * part_size + ti];
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[g][j] += p * bf2f((uint16_t)cur[u][j]);
        }
      }
    }
  }
  // reduce over the 4 token sub-lanes of the wave (tokens of wave w: w*4 + tg mod 4*NW)
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = acc[g][j];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      acc[g][j] = v;
    }
  __syncthreads();  // every wave is done reading `scores`, which `red` overlays
  if (tg == 0) {
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[(w * G + g) * D + ch * 8 + j] = acc[g][j];
  }
  __syncthreads();
  for (int i = tid; i < G * D; i += 64 * NW) {
    const int g = i / D, d = i % D;
    float v = 0.f;
#pragma unroll
    for (int wi = 0; wi < NW; ++wi) v += red[(wi * G + g) * D + d];
    const float inv = 1.f / stat[2 * g + 1];
    const int h = h0 + g;
    if (nparts == 1) {
      out[((int64_t)b * gridDim.y * G + h) * D + d] = f2bf(v * inv);
    } else {
      const int64_t slot = ((int64_t)b * gridDim.y * G + h) * max_parts + part;
      part_o[slot * D + d] = v * inv;
      if (d == 0) {
        part_ml[slot * 2] = stat[2 * g];
        part_ml[slot * 2 + 1] = stat[2 * g + 1];
      }
    }
  }
}

// grid: (B * Hq)   block: 128
__global__ __launch_bounds__(128) void decode_reduce_kernel(
    bf16_t* __restrict__ out, const float* __restrict__ part_o, const float* __restrict__ part_ml,
    const int* __restrict__ seq_lens, int hq, int part_size, int max_parts, int split_t,
    int split_min, int bs) {
  const int bh = blockIdx.x;
  const int b = bh / hq;
  const int len = seq_lens[b];
  if (len <= 0) return;
  const int pl = decode_part_len(len, part_size, split_t, split_min, bs);
  const int nparts = (len + pl - 1) / pl;
  if (nparts <= 1) return;
  const float* ml = part_ml + (int64_t)bh * max_parts * 2;
  float m = -INFINITY;
  for (int p = 0; p < nparts; ++p) m = fmaxf(m, ml[2 * p]);
  float tot = 0.f, acc = 0.f;
  const int d = threadIdx.x;
  for (int p = 0; p < nparts; ++p) {
    const float wgt = exp2f(ml[2 * p] - m) * ml[2 * p + 1];
    tot += wgt;
    acc += wgt * part_o[((int64_t)bh * max_parts + p) * D + d];
  }
  out[(int64_t)bh * D + d] = f2bf(acc / tot);
}

// ============================================================== prefill
__device__ __forceinline__ int kswz(int row, int ch) { return ch ^ (row & 15); }
__device__ __forceinline__ int vswz(int row, int ch) {
  return ch ^ (((row & 3) << 2) | ((row >> 2) & 3));
}

// grid: (Hq / HP, n_tiles)   block: 64*NW (NW waves x 16 query rows = a 16*NW-row
// query tile; every staged 64-key K/V tile feeds all NW waves)
// GQA head packing: each wave carries HP query heads of the same KV head for its
// 16 rows, so every K / V fragment read from LDS (and every K / V tile staged
// from HBM) feeds HP heads' MFMAs -- HP x fewer LDS bytes per FLOP and HP x
// fewer K/V tile loads than one head per block.
template <int BS, int HP, int NW>
__global__ __launch_bounds__(64 * NW) void prefill_attn_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc,
    const bf16_t* __restrict__ vc, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ q_start_loc, const int* __restrict__ seq_lens,
    const int* __restrict__ tile_seq, const int* __restrict__ tile_q0, int hkv, int64_t q_stride,
    int64_t out_stride, float scale_log2, float* __restrict__ lse_out,
    const int* __restrict__ kv_lens) {
  __shared__ __attribute__((aligned(16))) char lds[2 * 64 * 256];
  char* Kl = lds;
  char* Vl = lds + 64 * 256;

  const int h0 = blockIdx.x * HP, tile = blockIdx.y;
  const int hq = gridDim.x * HP;
  const int G = hq / hkv;
  const int kvh = h0 / G;
  const int s = tile_seq[tile], q0 = tile_q0[tile];
  const int qs = q_start_loc[s], qlen = q_start_loc[s + 1] - qs;
  const int ctx = seq_lens[s];
  const int off = ctx - qlen;  // absolute position of query row 0
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g4 = lane >> 4, c16 = lane & 15;
  const int* bt = block_tables + (int64_t)s * bt_stride;

  // query row owned by this lane (as the MFMA column)
  const int qr = q0 + w * 16 + c16;
  const bool row_ok = qr < qlen;
  const int qr_c = row_ok ? qr : qlen - 1;
  const int qpos = off + qr_c;
  short8 qf[HP][4];
#pragma unroll
  for (int hh = 0; hh < HP; ++hh) {
    const bf16_t* qrow = q + (int64_t)(qs + qr_c) * q_stride + (h0 + hh) * D;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
      qf[hh][kk] = *reinterpret_cast<const short8*>(qrow + kk * 32 + 8 * g4);
  }

  const int last_row = min(q0 + 16 * NW - 1, qlen - 1);
  // kv_lens (ring-attention blocks): keys >= klim are not part of this K/V block
  // even where the causal offset would admit them
  const int klim = kv_lens ? kv_lens[s] : 0x7fffffff;
  const int kv_end = min(off + last_row + 1, klim);  // keys [0, kv_end)
  const int ntiles = (kv_end + 63) / 64;
  const int min_qpos = off + q0;

  float m_run[HP], l_run[HP];
  float4v o[HP][8];
#pragma unroll
  for (int hh = 0; hh < HP; ++hh) {
    m_run[hh] = -INFINITY;
    l_run[hh] = 0.f;
#pragma unroll
    for (int mb = 0; mb < 8; ++mb) o[hh][mb] = float4v{0.f, 0.f, 0.f, 0.f};
  }

  constexpr int NCH = 16 / NW;  // 16-B chunks per thread per 64x128 tile
  short8 kreg[NCH], vreg[NCH];
  auto gload = [&](int t) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = i * 64 * NW + tid;
      const int row = c >> 4, ch = c & 15;
      const int key = t * 64 + row;
      if (key < kv_end) {
        const int64_t base = (((int64_t)bt[key / BS] * hkv + kvh) * BS + (key % BS)) * D + ch * 8;
        kreg[i] = *reinterpret_cast<const short8*>(kc + base);
        vreg[i] = *reinterpret_cast<const short8*>(vc + base);
      } else {
        kreg[i] = short8{0, 0, 0, 0, 0, 0, 0, 0};
        vreg[i] = short8{0, 0, 0, 0, 0, 0, 0, 0};
      }
    }
  };
  auto lwrite = [&]() {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = i * 64 * NW + tid;
      const int row = c >> 4, ch = c & 15;
      *reinterpret_cast<short8*>(Kl + row * 256 + 16 * kswz(row, ch)) = kreg[i];
      *reinterpret_cast<short8*>(Vl + row * 256 + 16 * vswz(row, ch)) = vreg[i];
    }
  };

  gload(0);
  lwrite();
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    if (t + 1 < ntiles) gload(t + 1);
    const int k0 = t * 64;
    // ---- S^T = K . Q^T  (each K fragment feeds HP heads)
    float4v sacc[HP][4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
#pragma unroll
      for (int hh = 0; hh < HP; ++hh) sacc[hh][nb] = float4v{0.f, 0.f, 0.f, 0.f};
      const int row = nb * 16 + c16;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        short8 a = *reinterpret_cast<const short8*>(Kl + row * 256 + 16 * kswz(row, kk * 4 + g4));
#pragma unroll
        for (int hh = 0; hh < HP; ++hh) sacc[hh][nb] = mfma16(a, qf[hh][kk], sacc[hh][nb]);
      }
    }
    const bool need_mask = (k0 + 63 > min_qpos) || (k0 + 63 >= ctx) || (k0 + 63 >= klim);
    short8 pb[HP][2];
#pragma unroll
    for (int hh = 0; hh < HP; ++hh) {
      float mloc = -INFINITY;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = sacc[hh][nb][r] * scale_log2;
          if (need_mask) {
            const int key = k0 + nb * 16 + g4 * 4 + r;
            if (key > qpos || key >= klim) v = -INFINITY;
          }
          sacc[hh][nb][r] = v;
          mloc = fmaxf(mloc, v);
        }
      mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
      mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
      const float m_new = fmaxf(m_run[hh], mloc);
      const float alpha = exp2f(m_run[hh] - m_new);
      float lsum = 0.f;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = exp2f(sacc[hh][nb][r] - m_new);
          sacc[hh][nb][r] = p;
          lsum += p;
        }
      lsum += __shfl_xor(lsum, 16, 64);
      lsum += __shfl_xor(lsum, 32, 64);
      l_run[hh] = l_run[hh] * alpha + lsum;
      m_run[hh] = m_new;
#pragma unroll
      for (int mb = 0; mb < 8; ++mb) o[hh][mb] *= alpha;
      // ---- P^T as B operand (k order permuted consistently with the V^T reads)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pb[hh][ks][j] = (short)f2bf(sacc[hh][2 * ks][j]);
          pb[hh][ks][4 + j] = (short)f2bf(sacc[hh][2 * ks + 1][j]);
        }
      }
    }
    // ---- O^T += V^T . P^T  (each V^T fragment feeds HP heads)
    const int qq = c16 >> 2, pp = c16 & 3;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int r1 = ks * 32 + g4 * 4 + qq;
      const int r2 = r1 + 16;
#pragma unroll
      for (int mb = 0; mb < 8; ++mb) {
        const int ch = 2 * mb + (pp >> 1);
        typedef short v4s __attribute__((ext_vector_type(4)));
        v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4s*)(Vl + r1 * 256 + 16 * vswz(r1, ch) + 8 * (pp & 1)));
        v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4s*)(Vl + r2 * 256 + 16 * vswz(r2, ch) + 8 * (pp & 1)));
        short8 a = short8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int hh = 0; hh < HP; ++hh) o[hh][mb] = mfma16(a, pb[hh][ks], o[hh][mb]);
      }
    }
    __syncthreads();
    if (t + 1 < ntiles) {
      lwrite();
      __syncthreads();
    }
  }

  if (row_ok) {
#pragma unroll
    for (int hh = 0; hh < HP; ++hh) {
      const float inv = 1.f / l_run[hh];
      bf16_t* orow = out + (int64_t)(qs + qr) * out_stride + (h0 + hh) * D;
#pragma unroll
      for (int mb = 0; mb < 8; ++mb) {
        uint2v pk;
        pk[0] = pack_bf2(o[hh][mb][0] * inv, o[hh][mb][1] * inv);
        pk[1] = pack_bf2(o[hh][mb][2] * inv, o[hh][mb][3] * inv);
        *reinterpret_cast<uint2v*>(orow + mb * 16 + g4 * 4) = pk;
      }
      // natural-log sum of exp of the scaled scores (m_run is in log2 units):
      // the merge statistic of ring attention / split-KV prefill
      if (lse_out && g4 == 0)
        lse_out[(int64_t)(qs + qr) * hq + h0 + hh] = (m_run[hh] + log2f(l_run[hh])) * 0.6931471805599453f;
    }
  }
}


// ----------------------------------------------------------- prefill, 32-row waves
// grid: (Hq / HB, n_tiles of 32 query rows)   block: 64 * HB
// One wave = 32 query rows of one head; the HB waves of a block are HB query
// heads of the same KV head over the SAME rows (GQA), so every 64-key K / V
// tile staged in LDS feeds HB heads and no wave of the block runs a causal
// tile the others skip.  Swapped products on 32x32x16 MFMA:
//   S^T = K . Q^T   lane (q = l&31, hi = l>>5) holds 32 of its row's 64 scores
//                   (keys half*32 + crow(r, hi), crow = (r&3) + 8(r>>2) + 4hi),
//                   so row max / sum are in-lane plus one xor-32 shuffle;
//   O^T += V^T . P^T  the P^T B operand of k-step s is the lane's OWN scores
//                   r = 8(s&1)+j of half s>>1 (no lane exchange): the k slots
//                   are permuted to those keys, and the V^T A operand reads the
//                   same keys -- two runs of 4 -- by ds_read_b64_tr_b16 from a
//                   row-major V image.
// Half the LDS bytes per MFMA of the 16-row kernel above (32 rows share every
// K / V fragment) and no cross-lane softmax beyond one shuffle per statistic.
__device__ __forceinline__ float16v mfma32(short8 a, short8 b, float16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// byte offset of 16-B chunk ch of row `row` in a [64][256 B] image: serves the
// ds_read_b128 row reads (K) and the transposed reads (V) conflict-free
__device__ __forceinline__ int img(int row, int ch) {
  return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

template <int BS, int HB>
__global__ __launch_bounds__(64 * HB, HB == 4 ? 2 : 1) void prefill_attn32_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc,
    const bf16_t* __restrict__ vc, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ q_start_loc, const int* __restrict__ seq_lens,
    const int* __restrict__ tile_seq, const int* __restrict__ tile_q0, int hkv, int64_t q_stride,
    int64_t out_stride, float scale_log2, float* __restrict__ lse_out,
    const int* __restrict__ kv_lens) {
  // two K | V stages (separate objects, so the compiler sees that fragment reads
  // of one stage cannot alias the other stage's in-flight LDS-DMA): the next
  // tile is written while this one is still read, one barrier per tile
  __shared__ __attribute__((aligned(16))) char st0[2 * 64 * 256];
  __shared__ __attribute__((aligned(16))) char st1[2 * 64 * 256];
  // the sequence's page indices for the first kMaxPages pages, staged once: a K/V
  // prefetch is then ONE global load deep instead of a page-table load followed
  // by the data load it feeds
  constexpr int kMaxPages = 1024;
  __shared__ int pg_lds[kMaxPages];

  const int hq = gridDim.x * HB;
  const int G = hq / hkv;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int h = blockIdx.x * HB + w;
  const int kvh = blockIdx.x * HB / G;
  const int tile = blockIdx.y;
  const int s = tile_seq[tile], q0 = tile_q0[tile];
  const int qs = q_start_loc[s], qlen = q_start_loc[s + 1] - qs;
  const int ctx = seq_lens[s];
  const int off = ctx - qlen;
  const int ql = lane & 31, hi = lane >> 5;
  const int* bt = block_tables + (int64_t)s * bt_stride;

  const int qr = q0 + ql;
  const bool row_ok = qr < qlen;
  const int qr_c = row_ok ? qr : qlen - 1;
  const int qpos = off + qr_c;
  short8 qf[8];
  {
    const bf16_t* qrow = q + (int64_t)(qs + qr_c) * q_stride + h * D;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
      qf[ks] = *reinterpret_cast<const short8*>(qrow + 16 * ks + 8 * hi);
  }
  const int last_row = min(q0 + 31, qlen - 1);
  const int klim = kv_lens ? kv_lens[s] : 0x7fffffff;
  const int kv_end = min(off + last_row + 1, klim);
  const int ntiles = (kv_end + 63) / 64;
  const int min_qpos = off + q0;

  const int npg = min((kv_end + BS - 1) / BS, kMaxPages);
  for (int i = tid; i < npg; i += 64 * HB) pg_lds[i] = bt[i];
  __syncthreads();

  // K / V tiles go global -> LDS by LDS-DMA (16 B per lane, 4 rows x 256 B per
  // wave instruction, no staging registers); the image's XOR is applied to the
  // per-lane SOURCE chunk (it is an involution).  Keys past kv_end re-read the
  // last valid key: their scores are masked, so P = 0 meets finite V rows.
  constexpr int NCH = 16 / HB;  // wave instructions per wave per 64-key tensor tile
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  auto dma = [&](int t, auto BUF) {
    char* Kl = decltype(BUF)::value ? st1 : st0;
    char* Vl = Kl + 64 * 256;
    int page[NCH];  // all page lookups before the first DMA issue
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int key = min(t * 64 + 4 * (w * NCH + i) + (lane >> 4), kv_end - 1);
      const int pi = key / BS;
      const int pl = pg_lds[pi < kMaxPages ? pi : 0];  // an LDS read, not a flat one
      page[i] = pi < kMaxPages ? pl : bt[pi];
    }
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int inst = w * NCH + i;
      const int row = 4 * inst + (lane >> 4), c = lane & 15;
      const int key = min(t * 64 + row, kv_end - 1);
      const int64_t base = (((int64_t)page[i] * hkv + kvh) * BS + (key % BS)) * D +
                           8 * (c ^ (((row & 3) << 2) | ((row >> 2) & 3)));
      __builtin_amdgcn_global_load_lds((const void*)(kc + base), (lds_ptr_t)(Kl + inst * 1024),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(vc + base), (lds_ptr_t)(Vl + inst * 1024),
                                       16, 0, 0);
    }
  };

  float m_run = -INFINITY, l_run = 0.f;
  float16v o[4];
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[db][r] = 0.f;

  // transposed-read lane roles: 16-lane group g = lane >> 4 covers d columns
  // 16 (g & 1) .. +15 of a 32-column block for k-slot half hi = g >> 1; lane
  // 4 qg + p of the group addresses key row qg, columns 4p .. 4p+3
  const int g = lane >> 4, qg = (lane & 15) >> 2, pp = lane & 3;

  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, 1>;
  dma(0, B0{});
  __syncthreads();  // vmcnt(0) + barrier: every wave's part of tile 0 landed
  // one tile on stage BUF while the next one's DMA fills the other stage; the
  // loop is unrolled by the two stages so every LDS address is a compile-time
  // offset from `lds` -- with a runtime stage index hipcc cannot tell the
  // fragment reads from the in-flight DMA's target and drains it (vmcnt(0))
  // before the first read, which serialises the prefetch
  auto body = [&](int t, auto BUF) {
    constexpr int buf = decltype(BUF)::value;
    // the other stage was last read in tile t-1, before the previous barrier
    if (t + 1 < ntiles) dma(t + 1, std::integral_constant<int, 1 - buf>{});
    const char* Kl = buf ? st1 : st0;
    const char* Vl = Kl + 64 * 256;
    const int k0 = t * 64;
    float16v sacc[2];
#pragma unroll
    for (int half = 0; half < 2; ++half) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[half][r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const short8 a = *reinterpret_cast<const short8*>(Kl + img(half * 32 + ql, 2 * ks + hi));
        sacc[half] = mfma32(a, qf[ks], sacc[half]);
      }
    }
    // causal / block mask only on tiles that reach past this wave's first query
    // (a wave-uniform branch): keys past `lim` (relative to k0) score -inf.
    // Scores stay unscaled here; the scale rides the exponent's FMA.
    float mloc = -INFINITY;
    if (k0 + 63 > min(min_qpos, klim - 1)) {
      const int lim = min(qpos, klim - 1) - k0 - 4 * hi;
#pragma unroll
      for (int half = 0; half < 2; ++half)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float v =
              half * 32 + (r & 3) + 8 * (r >> 2) > lim ? -INFINITY : sacc[half][r];
          sacc[half][r] = v;
          mloc = fmaxf(mloc, v);
        }
    } else {
#pragma unroll
      for (int half = 0; half < 2; ++half)
#pragma unroll
        for (int r = 0; r < 16; ++r) mloc = fmaxf(mloc, sacc[half][r]);
    }
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64)) * scale_log2;
    // lazy rescale: the running max moves only when a row's max grows by more
    // than 2^8 (P <= 256 is exact enough in bf16 / fp32); the O / l rescale is
    // skipped when no row of the wave moved (wave-uniform)
    const bool grow = mloc > m_run + 8.f;
    if (__builtin_amdgcn_ballot_w64(grow)) {
      const float m_new = grow ? mloc : m_run;
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);  // 0 on the first tile
      l_run *= alpha;
#pragma unroll
      for (int db = 0; db < 4; ++db) o[db] *= alpha;
      m_run = m_new;
    }
    // v_exp_f32 directly (arguments <= 8: underflow to 0 is the intended result)
    float lsum = 0.f;
#pragma unroll
    for (int half = 0; half < 2; ++half)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[half][r], scale_log2, -m_run));
        sacc[half][r] = p;
        lsum += p;
      }
    lsum += __shfl_xor(lsum, 32, 64);
    l_run += lsum;
    short8 pb[4];
#pragma unroll
    for (int st = 0; st < 4; ++st)
#pragma unroll
      for (int j = 0; j < 8; ++j)  // native RNE convert (v_cvt_pk_bf16_f32)
        pb[st][j] = __builtin_bit_cast(short, (__bf16)sacc[st >> 1][8 * (st & 1) + j]);
    typedef short v4s __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      // keys of k-step st for slot half g >> 1: (st>>1)*32 + 16(st&1) + 4(g>>1) + {0..3, 8..11}
      const int kb = (st >> 1) * 32 + 16 * (st & 1) + 4 * (g >> 1) + qg;
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const int ch = db * 4 + 2 * (g & 1) + (pp >> 1);
        v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4s*)(Vl + img(kb, ch) + 8 * (pp & 1)));
        v4s hv = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4s*)(Vl + img(kb + 8, ch) + 8 * (pp & 1)));
        const short8 a = __builtin_shufflevector(lo, hv, 0, 1, 2, 3, 4, 5, 6, 7);  // concat
        o[db] = mfma32(a, pb[st], o[db]);
      }
    }
    __syncthreads();  // tile t+1's DMA landed (vmcnt(0)) and tile t is read by all
  };
  for (int t = 0; t < ntiles; t += 2) {
    body(t, B0{});
    if (t + 1 < ntiles) body(t + 1, B1{});
  }

  if (row_ok) {
    const float inv = 1.f / l_run;
    bf16_t* orow = out + (int64_t)(qs + qr) * out_stride + h * D;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        uint2v pk;
        pk[0] = pack_bf2(o[db][4 * m] * inv, o[db][4 * m + 1] * inv);
        pk[1] = pack_bf2(o[db][4 * m + 2] * inv, o[db][4 * m + 3] * inv);
        *reinterpret_cast<uint2v*>(orow + db * 32 + 8 * m + 4 * hi) = pk;
      }
    if (lse_out && hi == 0)
      lse_out[(int64_t)(qs + qr) * hq + h] = (m_run + log2f(l_run)) * 0.6931471805599453f;
  }
}

}  // namespace

extern "C" {

// workspace: part_o [B*Hq*max_parts*128] f32, part_ml [B*Hq*max_parts*2] f32
int omnia_decode_attention(void* out, float* part_o, float* part_ml, const void* q,
                           const void* k_cache, const void* v_cache, const int* block_tables,
                           int bt_stride, const int* seq_lens, int B, int hq, int hkv,
                           int head_dim, int block_size, int64_t q_stride, int part_size,
                           int max_parts, float scale, int split_t, int split_min,
                           hipStream_t s) {
  if (head_dim != 128) return -1;
  if (part_size % 64 || part_size % block_size) return -2;
  if (split_t > 0 && (split_min <= 0 || split_t > max_parts)) return -5;
  if (B == 0) return 0;
  const int G = hq / hkv;
  const float scale_log2 = scale * 1.4426950408889634f;
  // OMNIA_DECODE_UG = 1 / 8 selects the single-group / 8-group K schedule
  // (A/B measurements; read per call)
  const char* ug_e = getenv("OMNIA_DECODE_UG");
  const int ug = ug_e && atoi(ug_e) == 1 ? 1 : (ug_e && atoi(ug_e) == 8 ? 8 : 4);
  // waves per workgroup: with many (sequence, kv head, partition) workgroups a
  // 4-wave group (90+ VGPRs -> 5 groups per CU) leaves ~2048 groups in two
  // uneven rounds; 2-wave groups keep every group of a 256-sequence batch
  // resident at once (16 waves / CU, one score tile of LDS each) and stream
  // the same bytes with the whole batch's loads in flight.  OMNIA_DECODE_NW
  // = 2 / 4 forces one (A/B, and the numerics tests cover both; read per call).
  const char* nw_e = getenv("OMNIA_DECODE_NW");
  const int nw_env = nw_e ? atoi(nw_e) : 0;
  const int64_t groups = (int64_t)B * hkv * max_parts;
  const int nw = nw_env == 2 || nw_env == 4 ? nw_env : (groups >= 1024 ? 2 : 4);
  // V rows in flight per lane in phase 3 (OMNIA_DECODE_U = 4 / 8, read per call)
  const char* u_e = getenv("OMNIA_DECODE_U");
  const int uv = u_e && atoi(u_e) == 8 ? 8 : 4;
  dim3 grid(B, hkv, max_parts), block(64 * nw);
  const size_t tile = (size_t)G * part_size > (size_t)nw * G * D ? (size_t)G * part_size
                                                                  : (size_t)nw * G * D;
  const size_t lds = 64 + tile * 4 + (part_size / block_size) * 4;
#define OMNIA_DEC_UG(GG, BB, UU, NN, VV)                                                       \
  decode_attn_kernel<GG, BB, UU, NN, VV><<<grid, block, lds, s>>>(                            \
      (bf16_t*)out, part_o, part_ml, (const bf16_t*)q, (const bf16_t*)k_cache,               \
      (const bf16_t*)v_cache, block_tables, bt_stride, seq_lens, hkv, q_stride, part_size,   \
      max_parts, scale_log2, split_t, split_min)
#define OMNIA_DEC_NW(GG, BB, UU, VV) \
  do { if (nw == 2) OMNIA_DEC_UG(GG, BB, UU, 2, VV); else OMNIA_DEC_UG(GG, BB, UU, 4, VV); } while (0)
#define OMNIA_DEC(GG, BB)                          \
  do {                                             \
    if (ug == 1) OMNIA_DEC_NW(GG, BB, 1, 4);       \
    else if (ug == 8) OMNIA_DEC_NW(GG, BB, 8, 8);  \
    else if (uv == 8) OMNIA_DEC_NW(GG, BB, 4, 8);  \
    else OMNIA_DEC_NW(GG, BB, 4, 4);               \
  } while (0)
#define OMNIA_DEC_BS(GG)                                \
  if (block_size == 16) OMNIA_DEC(GG, 16);              \
  else if (block_size == 32) OMNIA_DEC(GG, 32);         \
  else if (block_size == 64) OMNIA_DEC(GG, 64);         \
  else return -3;
  if (G == 1) { OMNIA_DEC_BS(1) }
  else if (G == 2) { OMNIA_DEC_BS(2) }
  else if (G == 4) { OMNIA_DEC_BS(4) }
  else if (G == 8) { OMNIA_DEC_BS(8) }
  else return -4;
#undef OMNIA_DEC_BS
#undef OMNIA_DEC
#undef OMNIA_DEC_NW
#undef OMNIA_DEC_UG
  if (max_parts > 1)
    decode_reduce_kernel<<<B * hq, 128, 0, s>>>((bf16_t*)out, part_o, part_ml, seq_lens, hq,
                                                part_size, max_parts, split_t, split_min,
                                                block_size);
  return (int)hipGetLastError();
}

int omnia_prefill_attention(void* out, const void* q, const void* k_cache, const void* v_cache,
                            const int* block_tables, int bt_stride, const int* q_start_loc,
                            const int* seq_lens, const int* tile_seq, const int* tile_q0,
                            int n_tiles, int hq, int hkv, int head_dim, int block_size,
                            int64_t q_stride, int64_t out_stride, float scale, int hp_req, int q_tile,
                            float* lse_out, const int* kv_lens, hipStream_t s) {
  if (head_dim != 128) return -1;
  if (hq % hkv) return -2;
  if (n_tiles == 0) return 0;
  const float scale_log2 = scale * 1.4426950408889634f;
  // heads per wave (GQA packing) and waves per block (query tile = 16 * nw rows)
  const int G = hq / hkv;
  static const int env_hp = getenv("OMNIA_PREFILL_HP") ? atoi(getenv("OMNIA_PREFILL_HP")) : 0;
  int hp = hp_req > 0 ? hp_req : env_hp > 0 ? env_hp : 1;
  if (hp != 1 && hp != 2 && hp != 4) return -5;
  if (G % hp) hp = 1;
  if (q_tile == 32) {
    // 32-row waves, HB heads of one KV head per block (prefill_attn32_kernel)
    const int hb = G % 4 == 0 ? 4 : G % 2 == 0 ? 2 : 1;
    dim3 grid32(hq / hb, n_tiles), block32(64 * hb);
#define OMNIA_PRE32(BB, HH)                                                                  \
  prefill_attn32_kernel<BB, HH><<<grid32, block32, 0, s>>>(                                  \
      (bf16_t*)out, (const bf16_t*)q, (const bf16_t*)k_cache, (const bf16_t*)v_cache,        \
      block_tables, bt_stride, q_start_loc, seq_lens, tile_seq, tile_q0, hkv, q_stride,      \
      out_stride, scale_log2, lse_out, kv_lens)
#define OMNIA_PRE32_HB(BB)                 \
  if (hb == 4) OMNIA_PRE32(BB, 4);         \
  else if (hb == 2) OMNIA_PRE32(BB, 2);    \
  else OMNIA_PRE32(BB, 1);
    if (block_size == 16) { OMNIA_PRE32_HB(16) }
    else if (block_size == 32) { OMNIA_PRE32_HB(32) }
    else if (block_size == 64) { OMNIA_PRE32_HB(64) }
    else return -3;
#undef OMNIA_PRE32_HB
#undef OMNIA_PRE32
    return (int)hipGetLastError();
  }
  const int nw = q_tile / 16;
  if (q_tile != 64 && q_tile != 128) return -6;
  if (nw == 8 && hp != 1) return -7;
  dim3 grid(hq / hp, n_tiles), block(64 * nw);
#define OMNIA_PRE(BB, HH, NN)                                                                \
  prefill_attn_kernel<BB, HH, NN><<<grid, block, 0, s>>>(                                    \
      (bf16_t*)out, (const bf16_t*)q, (const bf16_t*)k_cache, (const bf16_t*)v_cache,        \
      block_tables, bt_stride, q_start_loc, seq_lens, tile_seq, tile_q0, hkv, q_stride,      \
      out_stride, scale_log2, lse_out, kv_lens)
#define OMNIA_PRE_HP(BB)                              \
  if (nw == 8) OMNIA_PRE(BB, 1, 8);                   \
  else if (hp == 4) OMNIA_PRE(BB, 4, 4);              \
  else if (hp == 2) OMNIA_PRE(BB, 2, 4);              \
  else OMNIA_PRE(BB, 1, 4);
  if (block_size == 16) { OMNIA_PRE_HP(16) }
  else if (block_size == 32) { OMNIA_PRE_HP(32) }
  else if (block_size == 64) { OMNIA_PRE_HP(64) }
  else return -3;
#undef OMNIA_PRE_HP
#undef OMNIA_PRE
  return (int)hipGetLastError();
}

}  // extern "C"
