// Prefill GEMM with fused epilogues on gfx950:  out = X[M, K] . W[N, K]^T  for
// prefill chunks (M = hundreds to 16K rows), bf16 operands, fp32 MFMA accumulate.
// SURVEY §2.4 K3 (QKV), K4/K5 (RoPE + paged KV write), K8 (O), K9 (SwiGLU),
// K10 (down), K2 (residual add + RMSNorm).
//
// Main loop: the 256x256x64 "8-phase ping-pong" schedule (cdna_hip_programming.md
// §5, "The 256² 8-phase template"; T1-T5):
//   * 512 threads = 8 waves, 2 (rows) x 4 (cols); 16x16x32 bf16 MFMA; each wave
//     owns a 64x32 piece of every 128x128 quadrant of the block tile (128x64 total,
//     128 fp32 accumulators per lane);
//   * a K-tile (64 k) is four 16 KB half-tiles: A0/A1 (rows 0-127 / 128-255) and
//     B0/B1 (weight rows 0-127 / 128-255), each filled by direct LDS-DMA
//     (global_load_lds_dwordx4, 2 per thread) with the bank XOR (chunk c of row r at
//     c ^ (r & 7)) applied to the per-lane SOURCE address and to the reads;
//   * two K-tile buffers (128 KB); one phase per quadrant Q(A0,B0) Q(A0,B1)
//     Q(A1,B1) Q(A1,B0), so every half-tile is dead two phases after its last
//     ds_read and is restaged right then: one half-tile is in flight per phase,
//     retired by a counted `s_waitcnt vmcnt(4)` at phases 3 and 7 (never 0 in the
//     loop), raw s_barrier (hipcc's __syncthreads() would drain the DMA);
//   * the two wave rows run one barrier apart (ping-pong): while one wave of a
//     SIMD issues its ds_reads and DMA, the other's 16 MFMAs run (no s_setprio:
//     measured slower here);
//   * XCD-aware block order (bijective remap) with 8 m-tiles per group so the
//     blocks resident on one XCD share W column tiles and X row tiles in its L2.
// Epilogues (the accumulators are staged as bf16 through LDS, then every thread
// owns whole 16-B row chunks, so the fused ops read and write coalesced rows):
//   EPI 0  out = rs[r] * acc                                  (plain / row-scaled)
//   EPI 1  out = silu(rs*g) * (rs*u),  W = [Wg; Wu]            (gate_up + SwiGLU)
//   EPI 2  residual += acc  (in place), ss_out[r][tile] = sum of squares of the
//          new bf16 residual row slice                          (O / down)
//   EPI 3  rs-scaled QKV -> RoPE(q) to q_out, RoPE(k) and v to the paged KV cache
//   EPI 5  MoE grouped gate_up + SwiGLU: the 256-row tile's rows are expert-sorted
//          assignments (moe_align at 256-row segments), A rows gathered by token,
//          W = that segment's expert [Wg; Wu]; act written in sorted order
//   EPI 6  MoE grouped down: A = act (sorted order), W = the segment's expert,
//          each row scaled by its routing weight and scattered to Y[assignment]
//   EPI 4  split-K partial: block (m-tile, n-tile, k-slice ks) writes its K-slice's
//          fp32 sum, saturated to fp16, into slab ks of out[S][M][N]; the splitk.hip
//          consumers reduce the slabs (decode projections at M <= 256: one m-tile,
//          the K split fills the chip that N / 256 column tiles alone cannot)
// where rs[r] = rsqrt(sum_t ss_in[r][t] / d + eps): with the RMSNorm weight folded
// into W (W' = W * diag(w), models/llama.py fold_norms), RMSNorm(h) @ W^T ==
// rs * (h @ W'^T), so the normalisation rides the consumer's epilogue and the
// residual's sum of squares rides the producer's -- no RMSNorm, SwiGLU or RoPE
// launch exists in a prefill layer.
#include <type_traits>

#include "common.h"

using namespace omnia;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int BK = 64;
constexpr int HALF = 128 * BK;       // bf16 elements per half-tile (16 KB)
constexpr int MAIN = 8 * HALF;       // 2 buffers x 4 half-tiles (128 KB)
constexpr int SROW = 264;            // epilogue staging row stride (bf16): 528 B rows
constexpr int STAGE = 256 * SROW;    // 132 KB staging tile
constexpr int RS_OFF = STAGE > MAIN ? STAGE : MAIN;
constexpr int LDS_ELEMS = RS_OFF + 2 * 256;  // + 256 fp32 row scales

struct PArgs {
  void* out;            // EPI 0/1: bf16 [M, ldo]; EPI 2: residual bf16 [M, ldo]; EPI 3: q [M, ldo]
  const bf16_t* X;      // [M, K]
  const bf16_t* W;      // [N, K] ([2N, K] for EPI 1)
  int M, N, K, ldo;
  const float* ss_in;   // [M, ss_in_n] partial sums of squares (nullptr: no row scale)
  int ss_in_n;
  float inv_d, eps;
  float* ss_out;        // EPI 2: [M, N / 256]
  const int* positions;  // EPI 3
  const float* cos_sin;  // [max_pos, 128] = cos[64] | sin[64]
  bf16_t* k_cache;
  bf16_t* v_cache;       // [NB, hkv, BS, 128]
  const int64_t* slots;  // [M] (< 0: no KV write)
  int hq, hkv, block_size;
  int splits;            // EPI 4: K-slices (slabs)
  // EPI 5 / 6 (MoE grouped): sorted assignment ids [max_blocks * 256] (n_assign =
  // padding), per-256-row-segment expert, live segment count, routing weights
  const int* sorted;
  const int* blk_expert;
  const int* n_blocks;
  const float* route_w;
  int topk, n_assign, e_lo;
};

__device__ __forceinline__ float4v mfma16(short8 a, short8 b, float4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// two f32 -> packed fp16x2 (low = a), saturated to the fp16 range: a K-slice's
// partial beyond +-65504 stays finite (its slab sum then errs, never turns NaN)
__device__ __forceinline__ uint32_t pack_h2(float a, float b) {
  a = fminf(fmaxf(a, -65504.f), 65504.f);
  b = fminf(fmaxf(b, -65504.f), 65504.f);
  return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)a) |
         ((uint32_t)__builtin_bit_cast(uint16_t, (_Float16)b) << 16);
}

template <int EPI>
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  if constexpr (EPI == 4) return pack_h2(a, b);
  return pack_bf2(a, b);
}

__device__ __forceinline__ float16v mfma32(short8 a, short8 b, float16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

__device__ __forceinline__ float silu(float g) { return g * __builtin_amdgcn_rcpf(1.f + __expf(-g)); }

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// element offset of 16-B chunk `ch` of row `row` inside a half-tile
__device__ __forceinline__ int swz(int row, int ch) { return row * BK + ((ch ^ (row & 7)) << 3); }

// Epilogue copy-out shared by the 8-wave and 4-wave main loops: the block's
// 256 x TN tile is staged in LDS as bf16 ([256][SROW], rows of the tile), and
// every thread owns whole 16-B row chunks.
template <int EPI, int NT>
__device__ __forceinline__ void epi_out(const PArgs& p, const bf16_t* stg, int m0, int nt,
                                        int Mt, int ntn, int tid, int lane) {
  constexpr int TN = (EPI == 1 || EPI == 5) ? 128 : 256;
  if constexpr (EPI == 6) {
    // scatter the tile's live rows to their assignment rows of Y [n_assign, ldo]
    bf16_t* out = reinterpret_cast<bf16_t*>(p.out);
#pragma unroll 4
    for (int u = tid; u < 256 * 32; u += NT) {
      const int r = u >> 5, c = u & 31;
      const int f = p.sorted[m0 + r];
      if (f < p.n_assign)
        *reinterpret_cast<short8*>(out + (int64_t)f * p.ldo + (int64_t)nt * 256 + c * 8) =
            *reinterpret_cast<const short8*>(stg + r * SROW + c * 8);
    }
  } else if constexpr (EPI == 0 || EPI == 1 || EPI == 4 || EPI == 5) {
    // coalesced copy-out: TN/8 chunks per row (EPI 4: 16-bit fp16 chunks into
    // slab `ks`, whose base the caller folded into p.out)
    constexpr int CPR = TN / 8;
    bf16_t* out = reinterpret_cast<bf16_t*>(p.out);
#pragma unroll 4
    for (int u = tid; u < 256 * CPR; u += NT) {
      const int r = u / CPR, c = u - r * CPR;
      if (r < Mt)
        *reinterpret_cast<short8*>(out + (int64_t)(m0 + r) * p.ldo + (int64_t)nt * TN + c * 8) =
            *reinterpret_cast<const short8*>(stg + r * SROW + c * 8);
    }
  } else if constexpr (EPI == 2) {
    // residual += tile; 32 lanes per row (one 16-B chunk each) -> row sum of squares
    bf16_t* res = reinterpret_cast<bf16_t*>(p.out);
    const int c = lane & 31;
    const int rsub = (tid >> 5);  // NT/32 rows per pass
#pragma unroll 2
    for (int r0 = 0; r0 < 256; r0 += NT / 32) {
      const int r = r0 + rsub;
      float ss = 0.f;
      if (r < Mt) {
        bf16_t* rp = res + (int64_t)(m0 + r) * p.ldo + (int64_t)nt * 256 + c * 8;
        const short8 g = *reinterpret_cast<const short8*>(stg + r * SROW + c * 8);
        const short8 o = *reinterpret_cast<const short8*>(rp);
        short8 y;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint16_t h = f2bf(bf2f((uint16_t)o[j]) + bf2f((uint16_t)g[j]));
          const float hf = bf2f(h);
          ss += hf * hf;
          y[j] = (short)h;
        }
        *reinterpret_cast<short8*>(rp) = y;
      }
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
      if (c == 0 && r < Mt) p.ss_out[(int64_t)(m0 + r) * ntn + nt] = ss;
    }
  } else {
    // QKV: tile columns = heads 2nt, 2nt+1 of [q | k | v]; thread job = (row, head,
    // chunk pair c / c+8 = dims 8c..8c+7 and 64+8c..64+8c+7)
    bf16_t* qo = reinterpret_cast<bf16_t*>(p.out);
#pragma unroll 2
    for (int u = tid; u < 256 * 16; u += NT) {
      const int r = u >> 4, hh = (u >> 3) & 1, c = u & 7;
      if (r >= Mt) continue;
      const int t = m0 + r;
      const int head = nt * 2 + hh;  // global head index in [q heads | k heads | v heads]
      const short8 x1 = *reinterpret_cast<const short8*>(stg + r * SROW + hh * 128 + c * 8);
      const short8 x2 = *reinterpret_cast<const short8*>(stg + r * SROW + hh * 128 + 64 + c * 8);
      short8 o1 = x1, o2 = x2;
      if (head < p.hq + p.hkv) {
        const float* cs = p.cos_sin + (int64_t)p.positions[t] * 128;
        const float4v c0 = *reinterpret_cast<const float4v*>(cs + c * 8);
        const float4v c1 = *reinterpret_cast<const float4v*>(cs + c * 8 + 4);
        const float4v s0 = *reinterpret_cast<const float4v*>(cs + 64 + c * 8);
        const float4v s1 = *reinterpret_cast<const float4v*>(cs + 64 + c * 8 + 4);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float cj = j < 4 ? c0[j] : c1[j - 4], sj = j < 4 ? s0[j] : s1[j - 4];
          const float a = bf2f((uint16_t)x1[j]), b = bf2f((uint16_t)x2[j]);
          o1[j] = (short)f2bf(a * cj - b * sj);
          o2[j] = (short)f2bf(b * cj + a * sj);
        }
      }
      if (head < p.hq) {
        bf16_t* d = qo + (int64_t)t * p.ldo + head * 128 + c * 8;
        *reinterpret_cast<short8*>(d) = o1;
        *reinterpret_cast<short8*>(d + 64) = o2;
      } else {
        const int64_t slot = p.slots[t];
        if (slot >= 0) {
          const bool isk = head < p.hq + p.hkv;
          const int kh = isk ? head - p.hq : head - p.hq - p.hkv;
          const int64_t blk = slot / p.block_size, off = slot - blk * p.block_size;
          bf16_t* d = (isk ? p.k_cache : p.v_cache) +
                      ((blk * p.hkv + kh) * p.block_size + off) * 128 + c * 8;
          *reinterpret_cast<short8*>(d) = o1;
          *reinterpret_cast<short8*>(d + 64) = o2;
        }
      }
    }
  }
}

// VAR (tuning variants): bit 0 = no wave-row stagger, bit 1 = WITH s_setprio
// around the MFMA clusters, bits 2-3 = m-tiles per L2 group (8/4/16/32), bit 4 =
// 32x32x16 MFMA instead of 16x16x32 (same wave tile and LDS reads: a wave's
// 64x32 quadrant piece is 2 x 1 32x32 tiles, 8 MFMAs of twice the work per
// phase -- the chip can hold a different clock per MFMA shape)
template <int EPI, int VAR = 0>
__global__ __launch_bounds__(512, 2) void pgemm_kernel(PArgs p) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[LDS_ELEMS];
  constexpr int TN = (EPI == 1 || EPI == 5) ? 128 : 256;  // output columns per block tile
  constexpr bool MOE = EPI == 5 || EPI == 6;
  // EPI 4: the K-slices are extra "m-tiles" of the L2 grouping below (blocks of
  // one slice share its x slice, blocks of one column tile its W rows)
  const int S = EPI == 4 ? p.splits : 1;
  const int ntn = p.N / TN, mtn1 = (p.M + 255) >> 8, mtn = mtn1 * S;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  constexpr int GM = ((VAR >> 2) & 3) == 0 ? 8 : ((VAR >> 2) & 3) == 1 ? 4
                                           : ((VAR >> 2) & 3) == 2 ? 16 : 32;
  // s_setprio around the clusters measured 1.5-3.5 % SLOWER on every prefill shape
  // (profiles/r4/pgemm_variants.log), so the default build (VAR 0) leaves it out;
  // the wave-row stagger is worth ~15 % and stays
  constexpr bool STAGGER = !(VAR & 1), PRIO = (VAR & 2) != 0;
  constexpr bool M32 = (VAR & 16) != 0;
  const int per_group = GM * ntn;
  const int grp = bid / per_group, gm0 = grp * GM;
  const int gsz = mtn - gm0 < GM ? mtn - gm0 : GM;
  const int idx = bid - grp * per_group;
  const int vmt = gm0 + idx % gsz, nt = idx / gsz;
  const int ks = vmt / mtn1, mt = vmt - ks * mtn1;
  const int m0 = mt << 8, Mt = p.M - m0 < 256 ? p.M - m0 : 256;
  const int K = p.K, nk = K / S / BK;
  const int64_t kbase = (int64_t)ks * (K / S);
  // MoE: the grid is sized for the worst-case segment count (graph-safe, no host
  // sync); tiles past the live count leave, the whole block at once
  if constexpr (MOE) {
    if (mt >= *p.n_blocks) return;
  }
  const bf16_t* Wb = p.W;
  if constexpr (MOE)
    Wb += (int64_t)(p.blk_expert[mt] - p.e_lo) * (EPI == 5 ? 2 * p.N : p.N) * K;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;
  const int fr = lane & 15, fq = lane >> 4;

  // ---- LDS-DMA sources: instruction i of wave w fills half-tile rows 16w + 8i + lane/8,
  // LDS chunk lane%8 <- global chunk (lane%8) ^ (row & 7)
  const bf16_t* src[4][2];  // [A0, A1, B0, B1][i]
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 16 * w + 8 * i + (lane >> 3);
    const int gch = (lane & 7) ^ (row & 7);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      int ar = m0 + h * 128 + row;
      ar = ar < p.M ? ar : p.M - 1;  // rows past the chunk: clamped copies, never stored
      if constexpr (EPI == 5) {  // gather: the assignment's token row (padding: row 0)
        const int f = p.sorted[m0 + h * 128 + row];
        ar = f < p.n_assign ? f / p.topk : 0;
      }
      src[h][i] = p.X + (int64_t)ar * K + kbase + gch * 8;
      const int64_t br = (EPI == 1 || EPI == 5)
                             ? (int64_t)(h ? p.N : 0) + (int64_t)nt * 128 + row
                             : (int64_t)nt * 256 + h * 128 + row;
      src[2 + h][i] = Wb + br * K + kbase + gch * 8;
    }
  }
  auto issue = [&](int buf, auto HC, int kt) {
    constexpr int hidx = decltype(HC)::value;
    kt = kt < nk ? kt : nk - 1;  // past the end: reload the last tile into a dead slot
    bf16_t* dst = lds + (buf * 4 + hidx) * HALF + 16 * w * BK;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(src[hidx][i] + (int64_t)kt * BK),
                                       (lds_ptr_t)(dst + i * 512), 16, 0, 0);
  };

  float4v acc[2][2][4][2];   // 16x16 tiles: [qa][qb][m][n]
  float16v acc32[2][2][2];   // 32x32 tiles (M32): [qa][qb][m], n = 1
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      if constexpr (M32) {
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc32[a][b][m][r] = 0.f;
      } else {
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int n = 0; n < 2; ++n) acc[a][b][m][n] = {0.f, 0.f, 0.f, 0.f};
      }
    }

  // 16x16x32: af[m][ks] rows m*16 + fr, k chunk ks*4 + fq; 32x32x16: af[m][ks]
  // (m < 2, ks < 4) rows m*32 + (lane & 31), k chunk 2 ks + (lane >> 5)
  short8 af[4][2], bfr[2][2];
  const int l32 = lane & 31, h32 = lane >> 5;
  auto rdA = [&](int buf, int h) {
    const bf16_t* base = lds + (buf * 4 + h) * HALF;
    if constexpr (M32) {
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4)
          af[m * 2 + (k4 >> 1)][k4 & 1] = *reinterpret_cast<const short8*>(
              base + swz(wr * 64 + m * 32 + l32, k4 * 2 + h32));
    } else {
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          af[m][ks] = *reinterpret_cast<const short8*>(base + swz(wr * 64 + m * 16 + fr, ks * 4 + fq));
    }
  };
  auto rdB = [&](int buf, int h) {
    const bf16_t* base = lds + (buf * 4 + 2 + h) * HALF;
    if constexpr (M32) {
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4)
        bfr[k4 >> 1][k4 & 1] = *reinterpret_cast<const short8*>(
            base + swz(wc * 32 + l32, k4 * 2 + h32));
    } else {
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          bfr[n][ks] = *reinterpret_cast<const short8*>(base + swz(wc * 32 + n * 16 + fr, ks * 4 + fq));
    }
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;

  // phase P (0..7) of iteration `it` (K-tiles 2it in buffer 0, 2it+1 in buffer 1):
  //   quadrant q = P & 3 of buffer P >> 2: q0 (A0,B0) q1 (A0,B1) q2 (A1,B1) q3 (A1,B0)
  //   DMA: P0 A1(2it+1)->1  P1 B0(2it+1)->1  P2..P5 A0,B1,A1,B0(2it+2)->0
  //        P6,P7 A0,B1(2it+3)->1;   vmcnt(4) at P3 and P7
  auto phase = [&](auto PC, int it) {
    constexpr int P = decltype(PC)::value;
    constexpr int buf = P >> 2, q = P & 3;
    if constexpr (q == 0) {
      rdB(buf, 0);
      rdA(buf, 0);
    } else if constexpr (q == 1) {
      rdB(buf, 1);
    } else if constexpr (q == 2) {
      rdA(buf, 1);
    } else {
      rdB(buf, 0);
    }
    const int t0 = 2 * it;
    if constexpr (P == 0) issue(1, I1{}, t0 + 1);
    if constexpr (P == 1) issue(1, I2{}, t0 + 1);
    if constexpr (P == 2) issue(0, I0{}, t0 + 2);
    if constexpr (P == 3) issue(0, I3{}, t0 + 2);
    if constexpr (P == 4) issue(0, I1{}, t0 + 2);
    if constexpr (P == 5) issue(0, I2{}, t0 + 2);
    if constexpr (P == 6) issue(1, I0{}, t0 + 3);
    if constexpr (P == 7) issue(1, I3{}, t0 + 3);
    if constexpr (P == 3 || P == 7) wait_vm<4>();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    constexpr int qa = (q == 0 || q == 1) ? 0 : 1;
    constexpr int qb = (q == 0 || q == 3) ? 0 : 1;
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
    if constexpr (M32) {
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4)
#pragma unroll
        for (int m = 0; m < 2; ++m)
          acc32[qa][qb][m] = mfma32(af[m * 2 + (k4 >> 1)][k4 & 1], bfr[k4 >> 1][k4 & 1],
                                    acc32[qa][qb][m]);
    } else {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int n = 0; n < 2; ++n)
            acc[qa][qb][m][n] = mfma16(af[m][ks], bfr[n][ks], acc[qa][qb][m][n]);
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  // prologue: K-tile 0 -> buffer 0, A0/B1 of K-tile 1 -> buffer 1
  issue(0, I0{}, 0);
  issue(0, I2{}, 0);
  issue(0, I3{}, 0);
  issue(0, I1{}, 0);
  issue(1, I0{}, 1);
  issue(1, I3{}, 1);
  wait_vm<4>();
  __builtin_amdgcn_s_barrier();
  if (STAGGER && wr == 1) __builtin_amdgcn_s_barrier();  // second wave row one barrier behind
  const int nit = nk >> 1;
  for (int it = 0; it < nit; ++it) {
    phase(std::integral_constant<int, 0>{}, it);
    phase(std::integral_constant<int, 1>{}, it);
    phase(std::integral_constant<int, 2>{}, it);
    phase(std::integral_constant<int, 3>{}, it);
    phase(std::integral_constant<int, 4>{}, it);
    phase(std::integral_constant<int, 5>{}, it);
    phase(std::integral_constant<int, 6>{}, it);
    phase(std::integral_constant<int, 7>{}, it);
  }
  wait_vm<0>();  // the past-the-end reloads must land before LDS is reused
  if (STAGGER && wr == 0) __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_s_barrier();

  // ---------------------------------------------------------------- epilogue
  // lane rows: a*128 + wr*64 + m*16 + fq*4 + j ; cols: b*128 + wc*32 + n*16 + fr
  float* rs_lds = reinterpret_cast<float*>(lds + RS_OFF);
  const bool scaled = EPI == 6 || (EPI != 2 && p.ss_in != nullptr);
  if (scaled) {
    if (tid < 256) {
      if constexpr (EPI == 6) {  // row scale = the assignment's routing weight
        const int f = p.sorted[m0 + tid];
        rs_lds[tid] = f < p.n_assign ? p.route_w[f] : 0.f;
      } else {
        int r = m0 + tid;
        r = r < p.M ? r : p.M - 1;
        const float* s = p.ss_in + (int64_t)r * p.ss_in_n;
        float t = 0.f;
        for (int i = 0; i < p.ss_in_n; ++i) t += s[i];
        rs_lds[tid] = __builtin_amdgcn_rsqf(t * p.inv_d + p.eps);
      }
    }
    __syncthreads();
  }
  bf16_t* stg = lds;
  // write a 16x16 fragment's 4 rows x 1 col per lane as 2 rows x 2 cols (lane pairs
  // swap halves), i.e. two 4-byte LDS stores per fragment
  auto put = [&](int row0, int col, float v0, float v1, float v2, float v3) {
    const bool odd = fr & 1;
    const float s0 = odd ? v0 : v2, s1 = odd ? v1 : v3;
    const float r0 = __shfl_xor(s0, 1, 64), r1 = __shfl_xor(s1, 1, 64);
    uint32_t* d0;
    uint32_t* d1;
    uint32_t x0, x1;
    if (!odd) {
      d0 = reinterpret_cast<uint32_t*>(stg + (row0 + 0) * SROW + col);
      d1 = reinterpret_cast<uint32_t*>(stg + (row0 + 1) * SROW + col);
      x0 = pack2<EPI>(v0, r0);
      x1 = pack2<EPI>(v1, r1);
    } else {
      d0 = reinterpret_cast<uint32_t*>(stg + (row0 + 2) * SROW + col - 1);
      d1 = reinterpret_cast<uint32_t*>(stg + (row0 + 3) * SROW + col - 1);
      x0 = pack2<EPI>(r0, v2);
      x1 = pack2<EPI>(r1, v3);
    }
    *d0 = x0;
    *d1 = x1;
  };

  if constexpr (M32) {
    // 32x32 tiles: lane holds column l32 and rows 8g + 4 h32 + (0..3) of group
    // g = r >> 2 (r = 4g + j), i.e. four 4-row runs per tile
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row0 = a * 128 + wr * 64 + m * 32 + 8 * g + 4 * h32;
          float4v rs = {1.f, 1.f, 1.f, 1.f};
          if (scaled) rs = *reinterpret_cast<const float4v*>(rs_lds + row0);
          if constexpr (EPI == 1 || EPI == 5) {
            float v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
              v[j] = silu(acc32[a][0][m][4 * g + j] * rs[j]) * (acc32[a][1][m][4 * g + j] * rs[j]);
            put(row0, wc * 32 + l32, v[0], v[1], v[2], v[3]);
          } else {
#pragma unroll
            for (int b = 0; b < 2; ++b)
              put(row0, b * 128 + wc * 32 + l32, acc32[a][b][m][4 * g] * rs[0],
                  acc32[a][b][m][4 * g + 1] * rs[1], acc32[a][b][m][4 * g + 2] * rs[2],
                  acc32[a][b][m][4 * g + 3] * rs[3]);
          }
        }
  } else if constexpr (EPI == 1 || EPI == 5) {
    // gate (b = 0) and up (b = 1) of feature nt*128 + wc*32 + n*16 + fr in one lane
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int row0 = a * 128 + wr * 64 + m * 16 + fq * 4;
        float4v rs = {1.f, 1.f, 1.f, 1.f};
        if (scaled) rs = *reinterpret_cast<const float4v*>(rs_lds + row0);
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          float v[4];
#pragma unroll
          for (int j = 0; j < 4; ++j)
            v[j] = silu(acc[a][0][m][n][j] * rs[j]) * (acc[a][1][m][n][j] * rs[j]);
          put(row0, wc * 32 + n * 16 + fr, v[0], v[1], v[2], v[3]);
        }
      }
  } else {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int row0 = a * 128 + wr * 64 + m * 16 + fq * 4;
        float4v rs = {1.f, 1.f, 1.f, 1.f};
        if (scaled) rs = *reinterpret_cast<const float4v*>(rs_lds + row0);
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int n = 0; n < 2; ++n) {
            const float4v v = acc[a][b][m][n];
            put(row0, b * 128 + wc * 32 + n * 16 + fr, v[0] * rs[0], v[1] * rs[1], v[2] * rs[2],
                v[3] * rs[3]);
          }
      }
  }
  __syncthreads();

  if constexpr (EPI == 4) {
    PArgs q = p;
    q.out = reinterpret_cast<bf16_t*>(p.out) + (int64_t)ks * p.M * p.N;
    epi_out<4, 512>(q, stg, m0, nt, Mt, ntn, tid, lane);
  } else if constexpr (EPI == 5) {
    epi_out<1, 512>(p, stg, m0, nt, Mt, ntn, tid, lane);
  } else {
    epi_out<EPI, 512>(p, stg, m0, nt, Mt, ntn, tid, lane);
  }
}


// ---------------------------------------------------------------------------
// 4-wave schedule: one wave per SIMD, each wave a 128x128 quarter of the 256x256
// block tile (2 x 2 waves), 64 fp32 16x16 accumulators per lane (256 registers:
// the unified register file of a 1-wave-per-SIMD launch holds them beside the
// fragments).  Per K-tile (64 k) a wave issues 128 MFMAs back to back on
// independent accumulators; its LDS fragment reads for the NEXT half K-step are
// issued before the current 64 MFMAs (register double buffer), so the matrix
// core never waits on LDS.  Two LDS buffers; ONE barrier per K-tile, in the
// middle of it: after it, every wave has finished reading buffer t&1 and every
// wave's DMA of K-tile t+1 has landed, so the DMA of K-tile t+2 goes into
// buffer t&1 right there and has a whole K-tile of MFMA time to land.  The
// 8-wave ping-pong above parks ~26 % of its wave-cycles in its eight barriers
// per K-tile (profiles/r4/pgemm_pmc_summary.md); this schedule has one.
template <int EPI>
__global__ __launch_bounds__(256, 1) void pgemm4_kernel(PArgs p) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[LDS_ELEMS];
  constexpr int TN = EPI == 1 ? 128 : 256;
  const int S = EPI == 4 ? p.splits : 1;
  const int ntn = p.N / TN, mtn1 = (p.M + 255) >> 8, mtn = mtn1 * S;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  constexpr int GM = 8;
  const int per_group = GM * ntn;
  const int grp = bid / per_group, gm0 = grp * GM;
  const int gsz = mtn - gm0 < GM ? mtn - gm0 : GM;
  const int idx = bid - grp * per_group;
  const int vmt = gm0 + idx % gsz, nt = idx / gsz;
  const int ks = vmt / mtn1, mt = vmt - ks * mtn1;
  const int m0 = mt << 8, Mt = p.M - m0 < 256 ? p.M - m0 : 256;
  const int K = p.K, nk = K / S / BK;
  const int64_t kbase = (int64_t)ks * (K / S);

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int fr = lane & 15, fq = lane >> 4;

  // LDS-DMA: instruction i (0..3) of wave w fills half-tile rows 32w + 8i + lane/8;
  // the swizzled source chunk depends on lane/8 only, so instruction i reads
  // 8 i rows below instruction 0 (one base pointer per half-tile: 8 VGPRs, not 32)
  const bf16_t* src[4];
  {
    const int row = 32 * w + (lane >> 3);
    const int gch = (lane & 7) ^ (row & 7);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      int ar = m0 + h * 128 + row;
      src[h] = p.X + (int64_t)(ar < p.M ? ar : p.M - 1) * K + kbase + gch * 8;
      const int64_t br = EPI == 1 ? (int64_t)(h ? p.N : 0) + (int64_t)nt * 128 + row
                                  : (int64_t)nt * 256 + h * 128 + row;
      src[2 + h] = p.W + br * K + kbase + gch * 8;
    }
  }
  // A rows past the chunk: instruction i of an A half-tile may cross p.M (clamped
  // copies above only for i = 0) -> clamp per instruction below
  const int arow0 = m0 + 32 * w + (lane >> 3);
  auto issue_tile = [&](int buf, int kt) {
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      bf16_t* dst = lds + (buf * 4 + h) * HALF + 32 * w * BK;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int drow = 8 * i;
        if (h < 2) {  // rows past M: reload the last row (never stored)
          const int r0 = arow0 + h * 128;
          const int base = r0 < p.M ? r0 : p.M - 1;
          const int r = r0 + 8 * i;
          drow = (r < p.M ? r : p.M - 1) - base;
        }
        const int64_t off = (int64_t)kt * BK + (int64_t)drow * K;
        __builtin_amdgcn_global_load_lds((const void*)(src[h] + off),
                                         (lds_ptr_t)(dst + i * 512), 16, 0, 0);
      }
    }
  };

  // fragment rows: A of wave row wr; B of wave column wc (gate_up: n < 4 gate,
  // n >= 4 up of the SAME features, so silu(g) * u stays in one lane)
  // every EPI: n < 4 from B half-tile 0, n >= 4 from half-tile 1, wave column wc
  // owning columns wc*64 .. +64 of each half (compile-time half per fragment; a
  // runtime half measured worse register allocation: accumulators shuffled
  // through VGPRs inside the loop)
  auto browB = [&](int n) { return wc * 64 + (n & 3) * 16 + fr; };
  auto bhalf = [&](int n) { return n >> 2; };

  short8 fa[2][8], fb[2][8];
  auto read_frags = [&](int set, int buf, int ks) {
    const bf16_t* abase = lds + (buf * 4 + wr) * HALF;
#pragma unroll
    for (int m = 0; m < 8; ++m)
      fa[set][m] = *reinterpret_cast<const short8*>(abase + swz(m * 16 + fr, ks * 4 + fq));
#pragma unroll
    for (int n = 0; n < 8; ++n)
      fb[set][n] = *reinterpret_cast<const short8*>(lds + (buf * 4 + 2 + bhalf(n)) * HALF +
                                                    swz(browB(n), ks * 4 + fq));
  };

  float4v acc[8][8];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 8; ++n) acc[m][n] = {0.f, 0.f, 0.f, 0.f};
  auto mfma_all = [&](int set) {
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < 8; ++n) acc[m][n] = mfma16(fa[set][m], fb[set][n], acc[m][n]);
  };

  // prologue: K-tiles 0 and 1 in flight, wait for 0, first fragments
  issue_tile(0, 0);
  issue_tile(1, nk > 1 ? 1 : 0);
  wait_vm<16>();
  __builtin_amdgcn_s_barrier();
  read_frags(0, 0, 0);
  for (int t = 0; t < nk; ++t) {
    const int b = t & 1;
    // half 0: the 16 fragment reads of the second half K-step ride between the
    // 64 MFMAs of the first (one wave per SIMD: nobody else fills the MFMA pipe
    // while this wave issues memory instructions, so they are interleaved)
    read_frags(1, b, 1);
    mfma_all(0);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 LDS read
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // 4 MFMA
    }
    __builtin_amdgcn_sched_barrier(0);
    // every wave: its reads of buffer b retired and its DMA of K-tile t+1 landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // half 1: the next K-tile's 16 DMA and 16 first-half fragment reads between
    // the 64 MFMAs.  Unconditional (no control flow around the accumulators):
    // past the end the DMA reloads the last K-tile into the dead buffer and the
    // reads are unused
    issue_tile(b, t + 2 < nk ? t + 2 : nk - 1);
    read_frags(0, b ^ 1, 0);
    mfma_all(1);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // 1 VMEM (LDS-DMA)
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // 2 MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 LDS read
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // 2 MFMA
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  // pin the accumulators to AGPRs at the loop exit: otherwise the allocator keeps
  // some of them in VGPRs for the epilogue and shuffles them inside the loop
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 8; ++n) asm volatile("" : "+a"(acc[m][n]));
  wait_vm<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();  // every wave done with the ring before the staging tile reuses it

  // ---------------------------------------------------------------- epilogue
  float* rs_lds = reinterpret_cast<float*>(lds + RS_OFF);
  const bool scaled = EPI != 2 && p.ss_in != nullptr;
  if (scaled) {
    if (tid < 256) {
      int r = m0 + tid;
      r = r < p.M ? r : p.M - 1;
      const float* sp = p.ss_in + (int64_t)r * p.ss_in_n;
      float tt = 0.f;
      for (int i = 0; i < p.ss_in_n; ++i) tt += sp[i];
      rs_lds[tid] = __builtin_amdgcn_rsqf(tt * p.inv_d + p.eps);
    }
    __syncthreads();
  }
  bf16_t* stg = lds;
  auto put = [&](int row0, int col, float v0, float v1, float v2, float v3) {
    const bool odd = fr & 1;
    const float s0 = odd ? v0 : v2, s1 = odd ? v1 : v3;
    const float r0 = __shfl_xor(s0, 1, 64), r1 = __shfl_xor(s1, 1, 64);
    uint32_t* d0;
    uint32_t* d1;
    uint32_t x0, x1;
    if (!odd) {
      d0 = reinterpret_cast<uint32_t*>(stg + (row0 + 0) * SROW + col);
      d1 = reinterpret_cast<uint32_t*>(stg + (row0 + 1) * SROW + col);
      x0 = pack2<EPI>(v0, r0);
      x1 = pack2<EPI>(v1, r1);
    } else {
      d0 = reinterpret_cast<uint32_t*>(stg + (row0 + 2) * SROW + col - 1);
      d1 = reinterpret_cast<uint32_t*>(stg + (row0 + 3) * SROW + col - 1);
      x0 = pack2<EPI>(r0, v2);
      x1 = pack2<EPI>(r1, v3);
    }
    *d0 = x0;
    *d1 = x1;
  };
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int row0 = wr * 128 + m * 16 + fq * 4;
    float4v rs = {1.f, 1.f, 1.f, 1.f};
    if (scaled) rs = *reinterpret_cast<const float4v*>(rs_lds + row0);
    if constexpr (EPI == 1) {
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          v[j] = silu(acc[m][n][j] * rs[j]) * (acc[m][n + 4][j] * rs[j]);
        put(row0, wc * 64 + n * 16 + fr, v[0], v[1], v[2], v[3]);
      }
    } else {
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        const float4v v = acc[m][n];
        put(row0, (n >> 2) * 128 + wc * 64 + (n & 3) * 16 + fr, v[0] * rs[0], v[1] * rs[1],
            v[2] * rs[2], v[3] * rs[3]);
      }
    }
  }
  __syncthreads();
  if constexpr (EPI == 4) {
    PArgs q = p;
    q.out = reinterpret_cast<bf16_t*>(p.out) + (int64_t)ks * p.M * p.N;
    epi_out<4, 256>(q, stg, m0, nt, Mt, ntn, tid, lane);
  } else {
    epi_out<EPI, 256>(p, stg, m0, nt, Mt, ntn, tid, lane);
  }
}

// one workgroup (256 threads) per row: ss[r] = sum(x[r]^2) (layer-0 input of the
// folded-norm prefill path: the embedding rows have no producer epilogue)
__global__ __launch_bounds__(256) void row_sumsq_kernel(float* __restrict__ ss,
                                                        const bf16_t* __restrict__ x, int d,
                                                        int64_t stride) {
  __shared__ float red[4];
  const bf16_t* row = x + (int64_t)blockIdx.x * stride;
  float t = 0.f;
  for (int c = threadIdx.x * 8; c < d; c += 256 * 8) {
    const short8 v = *reinterpret_cast<const short8*>(row + c);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float f = bf2f((uint16_t)v[j]);
      t += f * f;
    }
  }
  t = block_sum(t, red);
  if (threadIdx.x == 0) ss[blockIdx.x] = t;
}

}  // namespace

extern "C" {

// Returns 0 on success, < 0 for a shape / argument the kernel does not cover
// (checked BEFORE any launch).
int omnia_pgemm_set_schedule(int sched);
int omnia_pgemm_variant(int variant, void* out, const void* X, const void* W, int M, int N,
                        int K, hipStream_t s);
int omnia_pgemm_splitk(void* parts, const void* X, const void* W, int M, int N, int K, int S,
                       int sched, hipStream_t s);
int omnia_pgemm_moe(int mode, void* out, const void* A, const void* W, const int* sorted,
                    const int* blk_expert, const int* n_blocks, const float* route_w, int K,
                    int N, int topk, int n_assign, int e_lo, int max_blocks, hipStream_t s);

static int g_pgemm_sched = 0;  // 0: 8-wave ping-pong, 1: 4-wave (one wave per SIMD)

int omnia_pgemm_set_schedule(int sched) {
  if (sched < 0 || sched > 1) return -1;
  g_pgemm_sched = sched;
  return 0;
}

int omnia_pgemm(int epi, void* out, const void* X, const void* W, int M, int N, int K, int ldo,
                const float* ss_in, int ss_in_n, float inv_d, float eps, float* ss_out,
                const int* positions, const float* cos_sin, void* k_cache, void* v_cache,
                const int64_t* slots, int hq, int hkv, int block_size, hipStream_t s) {
  if (epi < 0 || epi > 3) return -1;
  if (M < 1) return -2;
  if (K <= 0 || K % (2 * BK)) return -3;  // whole iterations of two K-tiles
  const int tn = epi == 1 ? 128 : 256;
  if (N <= 0 || N % tn) return -4;
  if ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W) |
       reinterpret_cast<uintptr_t>(out)) & 15)
    return -5;
  if (ldo % 8 || ldo < (epi == 3 ? hq * 128 : N)) return -6;
  if (ss_in != nullptr && ss_in_n < 1) return -7;
  if (epi == 2 && ss_out == nullptr) return -8;
  if (epi == 3) {
    if (!positions || !cos_sin || !k_cache || !v_cache || !slots || block_size < 1) return -9;
    // the epilogue works per head (a 256-column tile = heads 2nt, 2nt+1 of
    // [q | k | v]), so a tile may straddle the q / k / v boundaries: a TP shard's
    // single KV head (hkv * 128 = 128, Llama-3-70B at TP = 8) is fine
    if (hq < 1 || hkv < 1 || (hq + 2 * hkv) % 2) return -10;
    if (N != (hq + 2 * hkv) * 128) return -11;
    if ((reinterpret_cast<uintptr_t>(k_cache) | reinterpret_cast<uintptr_t>(v_cache)) & 15)
      return -12;
  }
  const int64_t blocks = (int64_t)((M + 255) / 256) * (N / tn);
  if (blocks > (1 << 30)) return -13;
  PArgs a{out, (const bf16_t*)X, (const bf16_t*)W, M, N, K, ldo, ss_in, ss_in_n, inv_d, eps,
          ss_out, positions, cos_sin, (bf16_t*)k_cache, (bf16_t*)v_cache, slots, hq, hkv,
          block_size, 1, nullptr, nullptr, nullptr, nullptr, 0, 0, 0};
  const dim3 grid((unsigned)blocks);
  if (g_pgemm_sched == 1) {
    switch (epi) {
      case 0: pgemm4_kernel<0><<<grid, 256, 0, s>>>(a); break;
      case 1: pgemm4_kernel<1><<<grid, 256, 0, s>>>(a); break;
      case 2: pgemm4_kernel<2><<<grid, 256, 0, s>>>(a); break;
      default: pgemm4_kernel<3><<<grid, 256, 0, s>>>(a); break;
    }
    return (int)hipGetLastError();
  }
  switch (epi) {
    case 0: pgemm_kernel<0><<<grid, 512, 0, s>>>(a); break;
    case 1: pgemm_kernel<1><<<grid, 512, 0, s>>>(a); break;
    case 2: pgemm_kernel<2><<<grid, 512, 0, s>>>(a); break;
    default: pgemm_kernel<3><<<grid, 512, 0, s>>>(a); break;
  }
  return (int)hipGetLastError();
}

// bare GEMM (EPI 0, no row scale) of a tuning variant: sweeps only
int omnia_pgemm_variant(int variant, void* out, const void* X, const void* W, int M, int N,
                        int K, hipStream_t s) {
  if (M < 1 || K <= 0 || K % (2 * BK) || N <= 0 || N % 256) return -1;
  PArgs a{out, (const bf16_t*)X, (const bf16_t*)W, M, N, K, N, nullptr, 0, 0.f, 0.f, nullptr,
          nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, 0, 1, nullptr, nullptr, nullptr,
          nullptr, 0, 0, 0};
  const dim3 grid((unsigned)(((M + 255) / 256) * (N / 256))), block(512);
  switch (variant) {
    case 0: pgemm_kernel<0, 0><<<grid, block, 0, s>>>(a); break;
    case 1: pgemm_kernel<0, 1><<<grid, block, 0, s>>>(a); break;
    case 2: pgemm_kernel<0, 2><<<grid, block, 0, s>>>(a); break;
    case 3: pgemm_kernel<0, 3><<<grid, block, 0, s>>>(a); break;
    case 4: pgemm_kernel<0, 4><<<grid, block, 0, s>>>(a); break;
    case 8: pgemm_kernel<0, 8><<<grid, block, 0, s>>>(a); break;
    case 12: pgemm_kernel<0, 12><<<grid, block, 0, s>>>(a); break;
    case 32: pgemm_kernel<0, 16><<<grid, block, 0, s>>>(a); break;   // 32x32x16 MFMA
    case 33: pgemm_kernel<0, 17><<<grid, block, 0, s>>>(a); break;
    case 34: pgemm_kernel<0, 18><<<grid, block, 0, s>>>(a); break;
    case 16: pgemm4_kernel<0><<<grid, 256, 0, s>>>(a); break;
    default: return -2;
  }
  return (int)hipGetLastError();
}

// split-K GEMM: parts[S][M][N] fp16, sum over s of parts[s] = X . W^T (EPI 4).
// `sched` 0 / 1 = the 8-wave / 4-wave main loop (independent of the prefill
// schedule switch: the decode table names the loop it measured).
int omnia_pgemm_splitk(void* parts, const void* X, const void* W, int M, int N, int K, int S,
                       int sched, hipStream_t s) {
  if (M < 1 || S < 1 || S > 16) return -1;
  if (K <= 0 || K % S || (K / S) % (2 * BK)) return -3;
  if (N <= 0 || N % 256) return -4;
  if ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W) |
       reinterpret_cast<uintptr_t>(parts)) & 15)
    return -5;
  const int64_t blocks = (int64_t)((M + 255) / 256) * (N / 256) * S;
  if (blocks > (1 << 30)) return -13;
  PArgs a{parts, (const bf16_t*)X, (const bf16_t*)W, M, N, K, N, nullptr, 0, 0.f, 0.f, nullptr,
          nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, 0, S, nullptr, nullptr, nullptr,
          nullptr, 0, 0, 0};
  if (sched == 1)
    pgemm4_kernel<4><<<dim3((unsigned)blocks), 256, 0, s>>>(a);
  else
    pgemm_kernel<4><<<dim3((unsigned)blocks), 512, 0, s>>>(a);
  return (int)hipGetLastError();
}

// MoE grouped GEMMs on the 256x256 tile (segments from omnia_moe_align with
// bm = 256).  mode 0: act [max_blocks*256, I] = SwiGLU(x[token] . W_gu[e]^T),
// x [T, d], W_gu [E_loc, 2I, d];  mode 1: Y[assignment] = w_route * act . W_dn[e]^T,
// act [max_blocks*256, I], W_dn [E_loc, d, I], Y [n_assign, d].
int omnia_pgemm_moe(int mode, void* out, const void* A, const void* W, const int* sorted,
                    const int* blk_expert, const int* n_blocks, const float* route_w, int K,
                    int N, int topk, int n_assign, int e_lo, int max_blocks, hipStream_t s) {
  if (mode < 0 || mode > 1 || max_blocks < 0 || topk < 1) return -1;
  if (K <= 0 || K % (2 * BK)) return -3;
  if (N <= 0 || N % (mode == 0 ? 128 : 256)) return -4;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(W) |
       reinterpret_cast<uintptr_t>(out)) & 15)
    return -5;
  if (!sorted || !blk_expert || !n_blocks || (mode == 1 && !route_w)) return -9;
  if (max_blocks == 0) return 0;
  const int64_t blocks = (int64_t)max_blocks * (N / (mode == 0 ? 128 : 256));
  if (blocks > (1 << 30)) return -13;
  PArgs a{out, (const bf16_t*)A, (const bf16_t*)W, max_blocks * 256, N, K, N, nullptr, 0, 0.f,
          0.f, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, 0, 1, sorted,
          blk_expert, n_blocks, route_w, topk, n_assign, e_lo};
  if (mode == 0)
    pgemm_kernel<5><<<dim3((unsigned)blocks), 512, 0, s>>>(a);
  else
    pgemm_kernel<6><<<dim3((unsigned)blocks), 512, 0, s>>>(a);
  return (int)hipGetLastError();
}

int omnia_row_sumsq(float* ss, const void* x, int rows, int d, int64_t stride, hipStream_t s) {
  if (d % 8 || rows < 0) return -1;
  if (rows == 0) return 0;
  row_sumsq_kernel<<<rows, 256, 0, s>>>(ss, (const bf16_t*)x, d, stride);
  return (int)hipGetLastError();
}

}  // extern "C"
