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
    const float* __restrict__ pres_pen, const float* __restrict__ rep_pen) {
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
                            hipStream_t s) {
  if (rows == 0) return 0;
  if (logits_is_bf16)
    sample_kernel<uint16_t><<<rows, kThreads, 0, s>>>(
        out_tok, out_logprob, (const uint16_t*)logits, row_stride, vocab, temperature, top_k,
        top_p, seeds, steps, counts, freq_pen, pres_pen, rep_pen);
  else
    sample_kernel<float><<<rows, kThreads, 0, s>>>(out_tok, out_logprob, (const float*)logits,
                                                   row_stride, vocab, temperature, top_k, top_p,
                                                   seeds, steps, counts, freq_pen, pres_pen,
                                                   rep_pen);
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
