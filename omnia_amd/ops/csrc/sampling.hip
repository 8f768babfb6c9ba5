// Fused token sampler -- one 1024-thread workgroup per sequence.
//
// Per row: penalties (frequency / presence / repetition from a per-sequence
// token-count table) -> greedy argmax when temperature == 0, otherwise
// temperature scaling -> exact top-k threshold (4-pass 8-bit radix select on
// the order-preserving key of the logits) -> exact top-p threshold (4-pass
// radix select on probability MASS, applied to the top-k survivors as
// PromptPack `parameters` define them) -> Gumbel-max draw from the survivors
// with a counter-based RNG keyed by (seed, step, token index).  Only the token
// id (and its log-prob under the temperature-scaled distribution) leave the
// GPU.  Rows stay resident in L2 across the passes (<= 512 KiB per row).
#include "common.h"

using namespace omnia;

namespace {

constexpr int kThreads = 1024;

__device__ __forceinline__ uint32_t fkey(float x) {
  const uint32_t u = __float_as_uint(x);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

template <typename T>
__device__ __forceinline__ float load_logit(const T* p, int i);
template <>
__device__ __forceinline__ float load_logit<float>(const float* p, int i) { return p[i]; }
template <>
__device__ __forceinline__ float load_logit<uint16_t>(const uint16_t* p, int i) {
  return bf2f(p[i]);
}

struct RowCtx {
  const int* counts;
  float freq, pres, rep, inv_t;
};

template <typename T>
__device__ __forceinline__ float value_at(const T* row, int i, const RowCtx& c) {
  float x = load_logit<T>(row, i);
  if (c.counts) {
    const int n = c.counts[i];
    if (n > 0) {
      if (c.rep != 1.f) x = x > 0.f ? x / c.rep : x * c.rep;
      x -= c.freq * (float)n + c.pres;
    }
  }
  return x * c.inv_t;
}

template <typename T>
__global__ __launch_bounds__(kThreads) void sample_kernel(
    int* __restrict__ out_tok, float* __restrict__ out_logprob, const T* __restrict__ logits,
    int64_t row_stride, int vocab, const float* __restrict__ temperature,
    const int* __restrict__ top_k, const float* __restrict__ top_p,
    const uint64_t* __restrict__ seeds, const int64_t* __restrict__ steps,
    int* __restrict__ counts, const float* __restrict__ freq_pen,
    const float* __restrict__ pres_pen, const float* __restrict__ rep_pen,
    int* __restrict__ tok_slots, const int64_t* __restrict__ dst) {
  __shared__ float red_f[kThreads / 64];
  __shared__ int red_i[kThreads / 64];
  __shared__ float red_z[kThreads / 64];
  __shared__ int hist[256];
  __shared__ float hmass[256];
  __shared__ uint32_t sh_prefix, sh_mask;
  __shared__ int sh_k;
  __shared__ float sh_target;

  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const T* lr = logits + (int64_t)row * row_stride;
  const float temp = temperature ? temperature[row] : 0.f;
  const bool greedy = !(temp > 0.f);
  RowCtx c;
  c.counts = counts ? counts + (int64_t)row * vocab : nullptr;
  c.freq = freq_pen ? freq_pen[row] : 0.f;
  c.pres = pres_pen ? pres_pen[row] : 0.f;
  c.rep = rep_pen ? rep_pen[row] : 1.f;
  c.inv_t = greedy ? 1.f : 1.f / temp;

  // ---- pass A: max, argmax and the partition function in ONE sweep (online
  // rescaling of the running sum), with 16-B loads when the row layout allows
  // (bf16 logits, no penalty table): the greedy path reads each logit once.
  float best = -INFINITY, z = 0.f;
  int besti = 0;
  auto visit = [&](float x, int i) {
    if (x == -INFINITY) return;  // masked token: no mass
    if (x > best) {
      z = z * __expf(best - x) + 1.f;  // exp(-inf) = 0 on the first hit
      best = x;
      besti = i;
    } else {
      z += __expf(x - best);
    }
  };
  const bool vec = sizeof(T) == 2 && c.counts == nullptr && (row_stride % 8) == 0 &&
                   (vocab % 8) == 0 && (reinterpret_cast<uintptr_t>(logits) & 15) == 0;
  if (vec) {
    const short8* lv = reinterpret_cast<const short8*>(lr);
    for (int ch = tid; ch < vocab / 8; ch += kThreads) {
      const short8 v = lv[ch];
#pragma unroll
      for (int j = 0; j < 8; ++j) visit(bf2f((uint16_t)v[j]) * c.inv_t, ch * 8 + j);
    }
  } else {
    for (int i = tid; i < vocab; i += kThreads) visit(value_at<T>(lr, i, c), i);
  }
  auto merge = [&](float ob, int oi, float oz) {
    const float m = fmaxf(best, ob);
    const float nz = (best == -INFINITY ? 0.f : z * __expf(best - m)) +
                     (ob == -INFINITY ? 0.f : oz * __expf(ob - m));
    if (ob > best || (ob == best && oi < besti)) besti = oi;
    best = m;
    z = nz;
  };
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
    merge(__shfl_xor(best, o, 64), __shfl_xor(besti, o, 64), __shfl_xor(z, o, 64));
  if (lane == 0) { red_f[wid] = best; red_i[wid] = besti; red_z[wid] = z; }
  __syncthreads();
  best = red_f[0];
  besti = red_i[0];
  z = red_z[0];
  for (int i = 1; i < kThreads / 64; ++i) merge(red_f[i], red_i[i], red_z[i]);
  const float M = best, Z = z;
  const int argm = besti;
  __syncthreads();

  if (greedy) {
    if (tid == 0) {
      out_tok[row] = argm;
      if (tok_slots) tok_slots[dst[row]] = argm;  // the sequence's device token slot
      if (out_logprob) out_logprob[row] = -__logf(Z);
      if (c.counts) counts[(int64_t)row * vocab + argm] += 1;
    }
    return;
  }

  // ---- top-k: exact k-th largest key by radix select
  uint32_t thr_key = 0;  // keep keys >= thr_key
  const int k = top_k ? top_k[row] : 0;
  if (k > 0 && k < vocab) {
    if (tid == 0) { sh_prefix = 0; sh_mask = 0; sh_k = k; }
    for (int shift = 24; shift >= 0; shift -= 8) {
      if (tid < 256) hist[tid] = 0;
      __syncthreads();
      const uint32_t pre = sh_prefix, msk = sh_mask;
      for (int i = tid; i < vocab; i += kThreads) {
        const uint32_t key = fkey(value_at<T>(lr, i, c));
        if ((key & msk) == pre) atomicAdd(&hist[(key >> shift) & 255], 1);
      }
      __syncthreads();
      if (tid == 0) {
        int kk = sh_k, b = 255;
        for (; b > 0; --b) {
          if (hist[b] >= kk) break;
          kk -= hist[b];
        }
        sh_k = kk;
        sh_prefix = pre | ((uint32_t)b << shift);
        sh_mask = msk | (255u << shift);
      }
      __syncthreads();
    }
    thr_key = sh_prefix;
  }

  // ---- top-p over the top-k survivors (mass renormalised to the survivors)
  const float p = top_p ? top_p[row] : 1.f;
  if (p < 1.f) {
    float zk = 0.f;
    for (int i = tid; i < vocab; i += kThreads) {
      const float x = value_at<T>(lr, i, c);
      if (fkey(x) >= thr_key) zk += __expf(x - M);
    }
    zk = block_sum(zk, red_f);
    if (tid == 0) { sh_prefix = 0; sh_mask = 0; sh_target = p * zk; }
    __syncthreads();
    for (int shift = 24; shift >= 0; shift -= 8) {
      if (tid < 256) hmass[tid] = 0.f;
      __syncthreads();
      const uint32_t pre = sh_prefix, msk = sh_mask;
      for (int i = tid; i < vocab; i += kThreads) {
        const float x = value_at<T>(lr, i, c);
        const uint32_t key = fkey(x);
        if (key >= thr_key && (key & msk) == pre)
          atomicAdd(&hmass[(key >> shift) & 255], __expf(x - M));
      }
      __syncthreads();
      if (tid == 0) {
        float tgt = sh_target;
        int b = 255;
        for (; b > 0; --b) {
          if (hmass[b] >= tgt) break;
          tgt -= hmass[b];
        }
        sh_target = tgt;
        sh_prefix = pre | ((uint32_t)b << shift);
        sh_mask = msk | (255u << shift);
      }
      __syncthreads();
    }
    if (sh_prefix > thr_key) thr_key = sh_prefix;
  }

  // ---- Gumbel-max draw among survivors
  const uint64_t seed = seeds ? seeds[row] : 0x5eedull;
  const uint64_t step = steps ? (uint64_t)steps[row] : 0ull;
  // (seed, step) only -- never the batch row -- so a seeded request draws the
  // same tokens whatever batch it lands in (pipelined vs synchronous, ragged finishes)
  const uint64_t rs = mix64(seed ^ (step * 0x9e3779b97f4a7c15ull));
  float gbest = -INFINITY, xsel = -INFINITY;
  int gi = argm;
  for (int i = tid; i < vocab; i += kThreads) {
    const float x = value_at<T>(lr, i, c);
    if (fkey(x) >= thr_key) {
      const float u = uniform01(rs, (uint64_t)i);
      const float g = x - __logf(-__logf(u));
      if (g > gbest) { gbest = g; gi = i; xsel = x; }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(gbest, o, 64);
    const int oi = __shfl_xor(gi, o, 64);
    const float ox = __shfl_xor(xsel, o, 64);
    if (ob > gbest || (ob == gbest && oi < gi)) { gbest = ob; gi = oi; xsel = ox; }
  }
  __syncthreads();
  __shared__ float red_x[kThreads / 64];
  if (lane == 0) { red_f[wid] = gbest; red_i[wid] = gi; red_x[wid] = xsel; }
  __syncthreads();
  if (tid == 0) {
    float bb = red_f[0], bx = red_x[0];
    int bi = red_i[0];
    for (int i = 1; i < kThreads / 64; ++i)
      if (red_f[i] > bb || (red_f[i] == bb && red_i[i] < bi)) {
        bb = red_f[i]; bi = red_i[i]; bx = red_x[i];
      }
    out_tok[row] = bi;
    if (tok_slots) tok_slots[dst[row]] = bi;
    if (out_logprob) out_logprob[row] = bx - M - __logf(Z);
    if (c.counts) counts[(int64_t)row * vocab + bi] += 1;
  }
}

}  // namespace

extern "C" int omnia_sample(int* out_tok, float* out_logprob, const void* logits,
                            int logits_is_bf16, int rows, int64_t row_stride, int vocab,
                            const float* temperature, const int* top_k, const float* top_p,
                            const uint64_t* seeds, const int64_t* steps, int* counts,
                            const float* freq_pen, const float* pres_pen, const float* rep_pen,
                            int* tok_slots, const int64_t* dst, hipStream_t s) {
  if (rows == 0) return 0;
  if (tok_slots && !dst) return -2;
  if (logits_is_bf16)
    sample_kernel<uint16_t><<<rows, kThreads, 0, s>>>(
        out_tok, out_logprob, (const uint16_t*)logits, row_stride, vocab, temperature, top_k,
        top_p, seeds, steps, counts, freq_pen, pres_pen, rep_pen, tok_slots, dst);
  else
    sample_kernel<float><<<rows, kThreads, 0, s>>>(out_tok, out_logprob, (const float*)logits,
                                                   row_stride, vocab, temperature, top_k, top_p,
                                                   seeds, steps, counts, freq_pen, pres_pen,
                                                   rep_pen, tok_slots, dst);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- K13 token mask
// logits[row, v] = -inf where bit v of mask[row] is clear (grammar-constrained rows;
// unconstrained rows carry all-ones masks).  One thread per (row, 32-token word):
// a 64-wide wave covers 2048 vocabulary entries with one mask load per lane.
namespace {
template <typename T>
__global__ void __launch_bounds__(256)
apply_token_mask_kernel(T* __restrict__ logits, int64_t row_stride, int vocab,
                        const uint32_t* __restrict__ mask, int words) {
  const int row = blockIdx.y;
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= words) return;
  const uint32_t m = mask[(int64_t)row * words + w];
  if (m == 0xffffffffu) return;
  T* lr = logits + (int64_t)row * row_stride + (int64_t)w * 32;
  const int n = min(32, vocab - w * 32);
  for (int i = 0; i < n; ++i)
    if (!((m >> i) & 1u)) {
      if constexpr (sizeof(T) == 2) lr[i] = (T)0xff80u;  // bf16 -inf
      else lr[i] = -INFINITY;
    }
}
}  // namespace

extern "C" int omnia_apply_token_mask(void* logits, int logits_is_bf16, int rows,
                                      int64_t row_stride, int vocab, const uint32_t* mask,
                                      int words, hipStream_t s) {
  if (rows == 0) return 0;
  dim3 grid((words + 255) / 256, rows);
  if (logits_is_bf16)
    apply_token_mask_kernel<uint16_t><<<grid, 256, 0, s>>>((uint16_t*)logits, row_stride, vocab,
                                                           mask, words);
  else
    apply_token_mask_kernel<float><<<grid, 256, 0, s>>>((float*)logits, row_stride, vocab, mask,
                                                        words);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- TP Gumbel winner
// Tensor-parallel sampling (parallel/tp_sampling.py): every TP rank reduces its
// vocabulary slice of each pure-temperature row to ONE Gumbel-max winner,
// argmax_v (logit_v / T - log(-log u_v)), with u a counter-based hash of
// (request seed, step, GLOBAL vocab id) -- murmur3 fmix32, bit-identical to
// tp_sampling.gumbel_uniform.  One pass over the bf16 logits, no noise tensor:
// a 256-thread workgroup per row, 8 contiguous bf16 (one 16-byte load) per lane
// per iteration.  Rows that are greedy or top-k / top-p filtered never read
// their logits (their winner is unused) and get (-inf, vocab_start).
// The (value, global id as float) pair is written straight into the candidate
// pack the ranks all-gather (columns col, col + 1 of a [B, ld] fp32 tensor).
namespace {
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  return h ^ (h >> 16);
}

__global__ void __launch_bounds__(256)
tp_gumbel_kernel(float* __restrict__ pack, int64_t ld, int col,
                 const uint16_t* __restrict__ logits, int64_t row_stride, int vocab,
                 int vocab_start, const float* __restrict__ temperature,
                 const int* __restrict__ top_k, const float* __restrict__ top_p,
                 const int64_t* __restrict__ seeds, const int64_t* __restrict__ steps) {
  const int row = blockIdx.x;
  const float t = temperature[row];
  float* dst = pack + (int64_t)row * ld + col;
  const bool pure = t > 0.f && (top_k == nullptr || top_k[row] <= 0) &&
                    (top_p == nullptr || top_p[row] >= 1.f);
  if (!pure) {
    if (threadIdx.x == 0) {
      dst[0] = -INFINITY;
      dst[1] = (float)vocab_start;
    }
    return;
  }
  const float tt = fmaxf(t, 1e-6f);
  const uint64_t sd = (uint64_t)seeds[row];
  const uint64_t st = steps ? (uint64_t)steps[row] : 0ull;
  uint32_t h = fmix32((uint32_t)sd ^ fmix32((uint32_t)(sd >> 32) ^ 0x68BC21EBu));
  h = fmix32(h ^ fmix32((uint32_t)st ^ 0x02E5BE93u));
  const uint16_t* lr = logits + (int64_t)row * row_stride;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  auto visit = [&](float x, int v) {
    const uint32_t r = fmix32(h ^ fmix32((uint32_t)(vocab_start + v) + 0x9E3779B9u));
    float u = (float)(((double)r + 0.5) * (1.0 / 4294967296.0));
    u = fminf(fmaxf(u, 1e-10f), 1.f - 1e-7f);
    const float g = x / tt - logf(-logf(u));
    if (g > best || (g == best && v < bi)) {
      best = g;
      bi = v;
    }
  };
  const bool vec = (row_stride % 8 == 0) && ((reinterpret_cast<uintptr_t>(logits) & 15) == 0);
  const int nv = vec ? vocab / 8 : 0;
  for (int c = threadIdx.x; c < nv; c += blockDim.x) {
    const uint4 q = reinterpret_cast<const uint4*>(lr)[c];
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      visit(__uint_as_float(w[j] << 16), c * 8 + 2 * j);
      visit(__uint_as_float(w[j] & 0xffff0000u), c * 8 + 2 * j + 1);
    }
  }
  for (int v = nv * 8 + threadIdx.x; v < vocab; v += blockDim.x) visit(bf2f(lr[v]), v);
  // wave argmax (ties -> lowest id), then across the 4 waves through LDS
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o);
    const int oi = __shfl_xor(bi, o);
    if (ob > best || (ob == best && oi < bi)) {
      best = ob;
      bi = oi;
    }
  }
  __shared__ float sb[4];
  __shared__ int si[4];
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sb[wave] = best;
    si[wave] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < 4; ++k)
      if (sb[k] > best || (sb[k] == best && si[k] < bi)) {
        best = sb[k];
        bi = si[k];
      }
    dst[0] = best;
    dst[1] = (float)(vocab_start + (bi == 0x7fffffff ? 0 : bi));
  }
}
}  // namespace

extern "C" int omnia_tp_gumbel(float* pack, int64_t ld, int col, const void* logits, int rows,
                               int64_t row_stride, int vocab, int vocab_start,
                               const float* temperature, const int* top_k, const float* top_p,
                               const int64_t* seeds, const int64_t* steps, hipStream_t s) {
  if (rows == 0) return 0;
  tp_gumbel_kernel<<<rows, 256, 0, s>>>(pack, ld, col, (const uint16_t*)logits, row_stride,
                                        vocab, vocab_start, temperature, top_k, top_p, seeds,
                                        steps);
  return (int)hipGetLastError();
}

// ------------------------------------------------ TP candidate pack + merge (decode)
// The tensor-parallel sampler on the GPU is two kernels around ONE all-gather
// (parallel/tp_sampling.py), with no framework ops in the captured decode graph:
//
// tp_pack (per rank, one 1024-thread workgroup per row of its vocab slice):
//   * greedy rows: the slice's arg-max (value, global id) -> cols 0, K;
//   * pure-temperature rows: the Gumbel-max winner of the slice (the tp_gumbel
//     hash above, bit-identical to tp_sampling.gumbel_uniform) -> cols 2K, 2K+1;
//   * top-k / top-p rows: the EXACT local top-K of the slice -- radix select on
//     the 16-bit order-preserving bf16 key (two 8-bit histogram passes), then an
//     index-ordered compaction (block prefix sums), so the candidate set and its
//     order are deterministic -- -> cols [0, K) values, [K, 2K) global ids; plus
//     the slice's softmax statistics of logits / T (max, sum exp) -> cols 2K+2,
//     2K+3, from which the merge gets the FULL-vocabulary partition function.
// tp_merge (every rank, same inputs -> same token; one 512-thread workgroup per
//   row) over the all-gathered packs [W][B][ld]:
//   * greedy: arg-max of the W slice maxima (ties -> lowest id);
//   * pure temperature: arg-max of the W Gumbel winners;
//   * filtered: the W*K candidates scaled by 1/T, bitonic-sorted in LDS, top-k
//     cut (ties at the k-th value kept), top-p cut against the full-vocabulary
//     mass (or the top-k survivors' mass when k > 0, as sample_kernel
//     renormalises), then the Gumbel-max draw with the SAME counter-based noise
//     as sample_kernel keyed by the GLOBAL token id -- so a filtered TP row draws
//     exactly the token the single-GPU fused sampler draws whenever the nucleus
//     / top-k set lies inside the candidates (top_k <= K);
//   * the token goes to out[row] and, fused, to tok_slots[dst[row]] (the
//     device token hand-off of pipelined decode).
namespace {
constexpr int kPackThreads = 1024;
constexpr int kMergeThreads = 512;

__device__ __forceinline__ uint32_t key16(uint32_t b) {
  return (b & 0x8000u) ? (~b & 0xffffu) : (b | 0x8000u);
}

// block-wide exclusive prefix sum of small ints; *total = block sum
__device__ __forceinline__ int block_excl_sum(int v, int* scratch, int* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  int inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  __syncthreads();  // previous readers of scratch are done
  if (lane == 63) scratch[wid] = inc;
  __syncthreads();
  int before = 0, tot = 0;
  for (int i = 0; i < nw; ++i) {
    const int c = scratch[i];
    before += i < wid ? c : 0;
    tot += c;
  }
  *total = tot;
  return before + inc - v;
}

// (value desc, id asc) arg-max merge
__device__ __forceinline__ void argmax_merge(float& bv, int& bi, float ov, int oi) {
  if (ov > bv || (ov == bv && oi < bi)) {
    bv = ov;
    bi = oi;
  }
}

__device__ __forceinline__ void block_argmax(float& bv, int& bi, float* sf, int* si) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) argmax_merge(bv, bi, __shfl_xor(bv, o, 64), __shfl_xor(bi, o, 64));
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) {
    sf[wid] = bv;
    si[wid] = bi;
  }
  __syncthreads();
  bv = sf[0];
  bi = si[0];
  for (int i = 1; i < nw; ++i) argmax_merge(bv, bi, sf[i], si[i]);
}

// element e of row `lr` (VEC: 8 consecutive per thread per tile)
template <bool VEC>
struct RowTile {
  static constexpr int E = VEC ? 8 : 1;
  __device__ __forceinline__ static void load(const uint16_t* lr, int idx0, int vocab,
                                              uint32_t (&b)[E], bool (&ok)[E]) {
    if (VEC) {
      if (idx0 < vocab) {  // vocab % 8 == 0: the whole vector is in the row
        const short8 v = *reinterpret_cast<const short8*>(lr + idx0);
#pragma unroll
        for (int j = 0; j < E; ++j) {
          b[j] = (uint16_t)v[j];
          ok[j] = true;
        }
      } else {
#pragma unroll
        for (int j = 0; j < E; ++j) {
          b[j] = 0;
          ok[j] = false;
        }
      }
    } else {
      ok[0] = idx0 < vocab;
      b[0] = ok[0] ? lr[idx0] : 0;
    }
  }
};

template <bool VEC>
__global__ void __launch_bounds__(kPackThreads)
tp_pack_kernel(float* __restrict__ pack, int64_t ld, int K, const uint16_t* __restrict__ logits,
               int64_t row_stride, int vocab, int vocab_start,
               const float* __restrict__ temperature, const int* __restrict__ top_k,
               const float* __restrict__ top_p, const int64_t* __restrict__ seeds,
               const int64_t* __restrict__ steps) {
  using RT = RowTile<VEC>;
  constexpr int E = RT::E;
  __shared__ int hist[256];
  __shared__ int iscr[kPackThreads / 64];
  __shared__ float fscr[kPackThreads / 64];
  __shared__ float fscr2[kPackThreads / 64];
  __shared__ int sh_a, sh_b;
  const int row = blockIdx.x, tid = threadIdx.x;
  const int tile = blockDim.x * E;
  const uint16_t* lr = logits + (int64_t)row * row_stride;
  float* dst = pack + (int64_t)row * ld;
  const float t = temperature[row];
  const bool greedy = !(t > 0.f);
  const bool filtered = !greedy && ((top_k != nullptr && top_k[row] > 0) ||
                                    (top_p != nullptr && top_p[row] < 1.f));
  // every column defined (the packs cross the all-gather whole)
  for (int c = tid; c < ld; c += blockDim.x)
    dst[c] = (c >= K && c < 2 * K) || c == 2 * K + 1 ? (float)vocab_start
             : c == 2 * K + 3                          ? 0.f
                                                       : -INFINITY;
  __syncthreads();

  if (greedy) {
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int i0 = tid * E; i0 < vocab; i0 += tile) {
      uint32_t b[E];
      bool ok[E];
      RT::load(lr, i0, vocab, b, ok);
#pragma unroll
      for (int j = 0; j < E; ++j)
        if (ok[j]) argmax_merge(bv, bi, bf2f((uint16_t)b[j]), i0 + j);
    }
    block_argmax(bv, bi, fscr, iscr);
    if (tid == 0) {
      dst[0] = bv;
      dst[K] = (float)(vocab_start + (bi == 0x7fffffff ? 0 : bi));
    }
    return;
  }
  const float inv_t = 1.f / fmaxf(t, 1e-6f);
  if (!filtered) {  // pure temperature: Gumbel-max winner (tp_gumbel's hash)
    const uint64_t sd = (uint64_t)seeds[row];
    const uint64_t st = steps ? (uint64_t)steps[row] : 0ull;
    uint32_t h = fmix32((uint32_t)sd ^ fmix32((uint32_t)(sd >> 32) ^ 0x68BC21EBu));
    h = fmix32(h ^ fmix32((uint32_t)st ^ 0x02E5BE93u));
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int i0 = tid * E; i0 < vocab; i0 += tile) {
      uint32_t b[E];
      bool ok[E];
      RT::load(lr, i0, vocab, b, ok);
#pragma unroll
      for (int j = 0; j < E; ++j) {
        if (!ok[j]) continue;
        const int v = i0 + j;
        const uint32_t r = fmix32(h ^ fmix32((uint32_t)(vocab_start + v) + 0x9E3779B9u));
        float u = (float)(((double)r + 0.5) * (1.0 / 4294967296.0));
        u = fminf(fmaxf(u, 1e-10f), 1.f - 1e-7f);
        argmax_merge(bv, bi, bf2f((uint16_t)b[j]) / fmaxf(t, 1e-6f) - logf(-logf(u)), v);
      }
    }
    block_argmax(bv, bi, fscr, iscr);
    if (tid == 0) {
      dst[2 * K] = bv;
      dst[2 * K + 1] = (float)(vocab_start + (bi == 0x7fffffff ? 0 : bi));
    }
    return;
  }

  // ---- filtered: softmax stats of x / T + high-byte histogram (one pass)
  for (int c = tid; c < 256; c += blockDim.x) hist[c] = 0;
  __syncthreads();
  float m = -INFINITY, s = 0.f;
  for (int i0 = tid * E; i0 < vocab; i0 += tile) {
    uint32_t b[E];
    bool ok[E];
    RT::load(lr, i0, vocab, b, ok);
#pragma unroll
    for (int j = 0; j < E; ++j) {
      if (!ok[j]) continue;
      atomicAdd(&hist[key16(b[j]) >> 8], 1);
      const float x = bf2f((uint16_t)b[j]) * inv_t;
      if (x == -INFINITY) continue;
      if (x > m) {
        s = s * __expf(m - x) + 1.f;
        m = x;
      } else {
        s += __expf(x - m);
      }
    }
  }
  // block merge of (m, s)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    const float nm = fmaxf(m, om);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    m = nm;
  }
  if ((tid & 63) == 0) {
    fscr[tid >> 6] = m;
    fscr2[tid >> 6] = s;
  }
  __syncthreads();  // also: hist complete
  if (tid == 0) {
    float M = fscr[0], S = fscr2[0];
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) {
      const float om = fscr[i], os = fscr2[i], nm = fmaxf(M, om);
      S = (M == -INFINITY ? 0.f : S * __expf(M - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
      M = nm;
    }
    dst[2 * K + 2] = M;
    dst[2 * K + 3] = S;
    // K-th largest key: its high byte, and how many keys lie strictly above it
    int cum = 0, bsel = 0;
    for (int bb = 255; bb >= 0; --bb) {
      if (cum + hist[bb] >= K) {
        bsel = bb;
        break;
      }
      cum += hist[bb];
    }
    sh_a = bsel;
    sh_b = cum;
  }
  __syncthreads();
  const uint32_t hi = (uint32_t)sh_a;
  const int above_hi = sh_b;
  for (int c = tid; c < 256; c += blockDim.x) hist[c] = 0;
  __syncthreads();
  for (int i0 = tid * E; i0 < vocab; i0 += tile) {
    uint32_t b[E];
    bool ok[E];
    RT::load(lr, i0, vocab, b, ok);
#pragma unroll
    for (int j = 0; j < E; ++j) {
      const uint32_t k = key16(b[j]);
      if (ok[j] && (k >> 8) == hi) atomicAdd(&hist[k & 255], 1);
    }
  }
  __syncthreads();
  if (tid == 0) {
    const int need = K - above_hi;
    int cum = 0, bsel = 0;
    for (int bb = 255; bb >= 0; --bb) {
      if (cum + hist[bb] >= need) {
        bsel = bb;
        break;
      }
      cum += hist[bb];
    }
    sh_a = (int)((hi << 8) | (uint32_t)bsel);  // threshold key
    sh_b = K - (above_hi + cum);               // keys == threshold to take
  }
  __syncthreads();
  const uint32_t thr = (uint32_t)sh_a;
  const int need_eq = sh_b;
  // ---- index-ordered compaction of the K selected (value, global id)
  int base_sel = 0, base_eq = 0;
  for (int t0 = 0; t0 < vocab && base_sel < K; t0 += tile) {
    const int i0 = t0 + tid * E;
    uint32_t b[E];
    bool ok[E];
    RT::load(lr, i0, vocab, b, ok);
    int n_eq = 0;
#pragma unroll
    for (int j = 0; j < E; ++j) n_eq += (ok[j] && key16(b[j]) == thr) ? 1 : 0;
    int tot_eq;
    const int eq_before = block_excl_sum(n_eq, iscr, &tot_eq);
    bool sel[E];
    int n_sel = 0, eq_seen = 0;
#pragma unroll
    for (int j = 0; j < E; ++j) {
      const uint32_t k = key16(b[j]);
      if (ok[j] && k > thr) {
        sel[j] = true;
      } else if (ok[j] && k == thr) {
        sel[j] = base_eq + eq_before + eq_seen < need_eq;
        ++eq_seen;
      } else {
        sel[j] = false;
      }
      n_sel += sel[j] ? 1 : 0;
    }
    int tot_sel;
    int pos = base_sel + block_excl_sum(n_sel, iscr, &tot_sel);
#pragma unroll
    for (int j = 0; j < E; ++j)
      if (sel[j] && pos < K) {
        dst[pos] = bf2f((uint16_t)b[j]);
        dst[K + pos] = (float)(vocab_start + i0 + j);
        ++pos;
      }
    base_eq += tot_eq;
    base_sel += tot_sel;
  }
}

// bitonic sort of kMergeThreads (value desc, id asc) pairs in LDS
__device__ __forceinline__ void bitonic_desc(float* v, int* id) {
  const int tid = threadIdx.x;
  for (int k = 2; k <= kMergeThreads; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      __syncthreads();
      const int p = tid ^ j;
      if (p > tid) {
        const bool up = (tid & k) == 0;  // this k-block sorted descending when up
        const float a = v[tid], c = v[p];
        const int ia = id[tid], ic = id[p];
        const bool a_first = a > c || (a == c && ia < ic);  // a precedes c in desc order
        if (up != a_first) {
          v[tid] = c;
          v[p] = a;
          id[tid] = ic;
          id[p] = ia;
        }
      }
    }
  }
  __syncthreads();
}

__global__ void __launch_bounds__(kMergeThreads)
tp_merge_kernel(int* __restrict__ out, int* __restrict__ tok_slots,
                const int64_t* __restrict__ dst_slot, const float* __restrict__ allp, int W,
                int B, int64_t ld, int K, const float* __restrict__ temperature,
                const int* __restrict__ top_k, const float* __restrict__ top_p,
                const int64_t* __restrict__ seeds, const int64_t* __restrict__ steps) {
  __shared__ float sv[kMergeThreads];
  __shared__ int sid[kMergeThreads];
  __shared__ float fscr[kMergeThreads / 64];
  __shared__ int iscr[kMergeThreads / 64];
  __shared__ int sh_keep;
  const int row = blockIdx.x, tid = threadIdx.x;
  const float t = temperature[row];
  const bool greedy = !(t > 0.f);
  const int k = top_k != nullptr ? top_k[row] : 0;
  const float p = top_p != nullptr ? top_p[row] : 1.f;
  const bool filtered = !greedy && (k > 0 || p < 1.f);
  auto pk = [&](int w) { return allp + ((int64_t)w * B + row) * ld; };
  int tok;
  if (!filtered) {
    const int vc = greedy ? 0 : 2 * K, ic = greedy ? K : 2 * K + 1;
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    if (tid < W) {
      const float* q = pk(tid);
      bv = q[vc];
      bi = (int)q[ic];
    }
    block_argmax(bv, bi, fscr, iscr);
    tok = bi == 0x7fffffff ? 0 : bi;
  } else {
    const float inv_t = 1.f / t;
    const int n = W * K;
    if (tid < n) {
      const float* q = pk(tid / K);
      const int j = tid - (tid / K) * K;
      const float x = q[j];
      sv[tid] = x == -INFINITY ? -INFINITY : x * inv_t;
      sid[tid] = (int)q[K + j];
    } else {
      sv[tid] = -INFINITY;
      sid[tid] = 0x7fffffff;
    }
    bitonic_desc(sv, sid);
    if (tid == 0) {
      const float M = sv[0];
      int nvalid = 0;
      while (nvalid < n && sv[nvalid] > -INFINITY) ++nvalid;
      int keep = nvalid;
      if (k > 0 && k < keep) {
        keep = k;
        while (keep < nvalid && sv[keep] == sv[k - 1]) ++keep;  // ties at the k-th kept
      }
      if (p < 1.f && keep > 0) {
        float Z = 0.f;
        if (k > 0) {
          for (int i = 0; i < keep; ++i) Z += __expf(sv[i] - M);
        } else {  // full-vocabulary mass from every rank's slice statistics
          for (int w = 0; w < W; ++w) {
            const float* q = pk(w);
            const float mw = q[2 * K + 2], sw = q[2 * K + 3];
            if (mw > -INFINITY) Z += sw * __expf(mw - M);
          }
        }
        const float target = p * Z;
        float cum = 0.f;
        int c = 0;
        for (; c < keep; ++c) {
          cum += __expf(sv[c] - M);
          if (cum >= target) break;
        }
        int keep2 = c < keep ? c + 1 : keep;
        while (keep2 < keep && sv[keep2] == sv[keep2 - 1]) ++keep2;
        keep = keep2;
      }
      sh_keep = keep;
    }
    __syncthreads();
    const int keep = sh_keep;
    const uint64_t seed = seeds ? (uint64_t)seeds[row] : 0x5eedull;
    const uint64_t step = steps ? (uint64_t)steps[row] : 0ull;
    const uint64_t rs = mix64(seed ^ (step * 0x9e3779b97f4a7c15ull));
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    if (tid < keep) {
      const float u = uniform01(rs, (uint64_t)sid[tid]);
      argmax_merge(bv, bi, sv[tid] - __logf(-__logf(u)), sid[tid]);
    }
    block_argmax(bv, bi, fscr, iscr);
    tok = bi == 0x7fffffff ? (keep > 0 ? sid[0] : 0) : bi;
  }
  if (tid == 0) {
    out[row] = tok;
    if (tok_slots != nullptr) tok_slots[dst_slot[row]] = tok;
  }
}
}  // namespace

extern "C" int omnia_tp_pack(float* pack, int64_t ld, int K, const void* logits, int rows,
                             int64_t row_stride, int vocab, int vocab_start,
                             const float* temperature, const int* top_k, const float* top_p,
                             const int64_t* seeds, const int64_t* steps, hipStream_t s) {
  if (rows == 0) return 0;
  if (K < 1 || K > vocab || ld < 2 * K + 4) return -1;
  const bool vec = (row_stride % 8) == 0 && (vocab % 8) == 0 &&
                   (reinterpret_cast<uintptr_t>(logits) & 15) == 0;
  if (vec)
    tp_pack_kernel<true><<<rows, kPackThreads, 0, s>>>(pack, ld, K, (const uint16_t*)logits,
                                                       row_stride, vocab, vocab_start,
                                                       temperature, top_k, top_p, seeds, steps);
  else
    tp_pack_kernel<false><<<rows, kPackThreads, 0, s>>>(pack, ld, K, (const uint16_t*)logits,
                                                        row_stride, vocab, vocab_start,
                                                        temperature, top_k, top_p, seeds, steps);
  return (int)hipGetLastError();
}

extern "C" int omnia_tp_merge(int* out, int* tok_slots, const int64_t* dst_slot, const float* allp,
                              int W, int B, int64_t ld, int K, const float* temperature,
                              const int* top_k, const float* top_p, const int64_t* seeds,
                              const int64_t* steps, hipStream_t s) {
  if (B == 0) return 0;
  if (W < 1 || K < 1 || W * K > kMergeThreads || ld < 2 * K + 4) return -1;
  tp_merge_kernel<<<B, kMergeThreads, 0, s>>>(out, tok_slots, dst_slot, allp, W, B, ld, K,
                                              temperature, top_k, top_p, seeds, steps);
  return (int)hipGetLastError();
}
