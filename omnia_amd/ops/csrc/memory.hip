// Memory-tier kernels for the in-node memory-api:
//   * mean_pool_l2  : masked mean-pool of an embedding model's last hidden
//                     states over each sequence + L2 normalisation -> fp32 vectors
//                     (replaces the remote embedding provider,
//                     reference internal/memory/embedding.go:36-105)
//   * cosine_scores : brute-force q . m over a workspace's bf16 unit vectors,
//                     fp32 accumulate (replaces pgvector's HNSW `<=>` scan,
//                     reference internal/memory/retrieve_multi_tier_hybrid.go:86-100)
//   * topk          : exact top-k per query by 8-bit radix select on the
//                     order-preserving uint32 image of the scores, then a
//                     bitonic sort of the k survivors in LDS.
// Vectors are stored normalised, so cosine similarity is a dot product and the
// scan is one pass over N*D*2 bytes of HBM (bandwidth bound).
#include "common.h"

using namespace omnia;

namespace {

// ------------------------------------------------------------ K17 mean-pool
// hidden: [T_total, D] bf16 (row stride `stride`), cu: [B+1] token offsets.
// grid (B), block 256; thread owns columns (i*256+tid)*8 .. +8 for i < VEC.
template <int VEC>
__global__ __launch_bounds__(256) void mean_pool_l2_kernel(float* __restrict__ out,
                                                           const bf16_t* __restrict__ h,
                                                           int64_t stride,
                                                           const int* __restrict__ cu, int D) {
  __shared__ float scratch[8];
  const int b = blockIdx.x;
  const int t0 = cu[b], t1 = cu[b + 1];
  float acc[VEC][8];
#pragma unroll
  for (int i = 0; i < VEC; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0.f;
  int t = t0;
  // two tokens per iteration: two independent 16-B loads in flight per chunk
  for (; t + 1 < t1; t += 2) {
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      const int c = (i * 256 + threadIdx.x) * 8;
      if (c < D) {
        const short8 a = *reinterpret_cast<const short8*>(h + (int64_t)t * stride + c);
        const short8 bb = *reinterpret_cast<const short8*>(h + (int64_t)(t + 1) * stride + c);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] += bf2f((uint16_t)a[j]) + bf2f((uint16_t)bb[j]);
      }
    }
  }
  if (t < t1) {
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      const int c = (i * 256 + threadIdx.x) * 8;
      if (c < D) {
        const short8 a = *reinterpret_cast<const short8*>(h + (int64_t)t * stride + c);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] += bf2f((uint16_t)a[j]);
      }
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VEC; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += acc[i][j] * acc[i][j];
  ss = block_sum(ss, scratch);
  // mean then normalise == normalise the sum (the 1/n cancels); empty -> zeros
  const float scale = (t1 > t0 && ss > 0.f) ? rsqrtf(ss) : 0.f;
  float* o = out + (int64_t)b * D;
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    const int c = (i * 256 + threadIdx.x) * 8;
    if (c < D) {
      float4v lo = {acc[i][0] * scale, acc[i][1] * scale, acc[i][2] * scale, acc[i][3] * scale};
      float4v hi = {acc[i][4] * scale, acc[i][5] * scale, acc[i][6] * scale, acc[i][7] * scale};
      *reinterpret_cast<float4v*>(o + c) = lo;
      *reinterpret_cast<float4v*>(o + c + 4) = hi;
    }
  }
}

// ------------------------------------------------------------ K18 scores
// Q: [NQ, D] fp32 staged in LDS; M: [N, D] bf16 rows.  8 lanes per row (the 8
// lanes read one contiguous 128 B span per step), 32 rows per 256-thread block
// per iteration, grid-stride over N.  valid (optional) masks tombstoned rows.
template <int NQ>
__global__ __launch_bounds__(256) void cosine_scores_kernel(float* __restrict__ scores,
                                                            const float* __restrict__ Q,
                                                            const bf16_t* __restrict__ M,
                                                            int64_t N, int D,
                                                            const uint8_t* __restrict__ valid) {
  extern __shared__ float qs[];  // [NQ][D]
  for (int i = threadIdx.x * 4; i < NQ * D; i += 256 * 4)
    *reinterpret_cast<float4v*>(qs + i) = *reinterpret_cast<const float4v*>(Q + i);
  __syncthreads();
  const int l8 = threadIdx.x & 7;
  const int grp = threadIdx.x >> 3;
  for (int64_t row = (int64_t)blockIdx.x * 32 + grp; row < N; row += (int64_t)gridDim.x * 32) {
    float acc[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[q] = 0.f;
    const bf16_t* mr = M + row * D;
    for (int c = l8 * 8; c < D; c += 64) {
      const short8 m = *reinterpret_cast<const short8*>(mr + c);
      float mf[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) mf[j] = bf2f((uint16_t)m[j]);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const float4v a = *reinterpret_cast<const float4v*>(qs + q * D + c);
        const float4v b = *reinterpret_cast<const float4v*>(qs + q * D + c + 4);
        acc[q] += a[0] * mf[0] + a[1] * mf[1] + a[2] * mf[2] + a[3] * mf[3] + b[0] * mf[4] +
                  b[1] * mf[5] + b[2] * mf[6] + b[3] * mf[7];
      }
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      float v = acc[q];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      acc[q] = v;
    }
    if (l8 == 0) {
      const bool ok = valid == nullptr || valid[row] != 0;
#pragma unroll
      for (int q = 0; q < NQ; ++q) scores[(int64_t)q * N + row] = ok ? acc[q] : -INFINITY;
    }
  }
}

// ------------------------------------------------------------ top-k
__device__ __forceinline__ uint32_t fkey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // monotone: larger float -> larger key
}

// one 1024-thread workgroup per query row of `scores` [NQ, N]; k <= 1024
__global__ __launch_bounds__(1024) void topk_kernel(int* __restrict__ out_idx,
                                                    float* __restrict__ out_val,
                                                    const float* __restrict__ scores, int64_t N,
                                                    int k) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t s_prefix, s_remaining, s_gt, s_eq;
  __shared__ uint32_t ckey[2048];
  __shared__ int cidx[2048];
  const float* row = scores + (int64_t)blockIdx.x * N;
  const int tid = threadIdx.x;
  uint32_t prefix = 0, mask = 0;
  uint32_t remaining = (uint32_t)k;  // rank (1-based) of the target among matching keys
  for (int shift = 24; shift >= 0; shift -= 8) {
    if (tid < 256) hist[tid] = 0;
    __syncthreads();
    for (int64_t i = tid; i < N; i += 1024) {
      const uint32_t key = fkey(row[i]);
      if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t acc = 0;
      int d = 255;
      for (; d > 0; --d) {
        if (acc + hist[d] >= remaining) break;
        acc += hist[d];
      }
      s_prefix = prefix | ((uint32_t)d << shift);
      s_remaining = remaining - acc;
    }
    __syncthreads();
    prefix = s_prefix;
    remaining = s_remaining;
    mask |= 255u << shift;
  }
  // prefix is now the k-th largest key T; (k - remaining) keys are > T.
  // Compaction in index order (ballot + per-wave prefix) so that among keys
  // equal to T the lowest indices are kept: results are deterministic.
  __shared__ uint32_t wgt[16], weq[16];
  if (tid == 0) { s_gt = 0; s_eq = 0; }
  __syncthreads();
  const uint32_t T = prefix;
  const uint32_t n_gt = (uint32_t)k - remaining;
  const int lane = tid & 63, w = tid >> 6;
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int64_t base = 0; base < N; base += 1024) {
    const int64_t i = base + tid;
    const uint32_t key = i < N ? fkey(row[i]) : 0u;
    const bool gt = i < N && key > T;
    const bool eq = i < N && key == T;
    const uint64_t bg = __ballot(gt), be = __ballot(eq);
    if (lane == 0) { wgt[w] = __popcll(bg); weq[w] = __popcll(be); }
    __syncthreads();
    uint32_t og = s_gt, oe = s_eq;
    for (int j = 0; j < w; ++j) { og += wgt[j]; oe += weq[j]; }
    if (gt) {
      const uint32_t p = og + __popcll(bg & lt_mask);
      ckey[p] = key;
      cidx[p] = (int)i;
    } else if (eq) {
      const uint32_t p = oe + __popcll(be & lt_mask);
      if (p < remaining) {
        ckey[n_gt + p] = key;
        cidx[n_gt + p] = (int)i;
      }
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t tg = 0, te = 0;
      for (int j = 0; j < 16; ++j) { tg += wgt[j]; te += weq[j]; }
      s_gt += tg;
      s_eq += te;
    }
    __syncthreads();
  }
  // bitonic sort (descending key, ascending index on ties) over pow2 >= k
  int n2 = 1;
  while (n2 < k) n2 <<= 1;
  for (int i = k + tid; i < n2; i += 1024) { ckey[i] = 0u; cidx[i] = 0x7fffffff; }
  __syncthreads();
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < n2; i += 1024) {
        const int j = i ^ stride;
        if (j > i) {
          const bool desc = (i & size) == 0;
          const uint32_t ki = ckey[i], kj = ckey[j];
          const int ii = cidx[i], ij = cidx[j];
          // "i before j" in the final order: larger key first, then smaller index
          const bool i_first = ki > kj || (ki == kj && ii < ij);
          if (desc != i_first) {
            ckey[i] = kj; ckey[j] = ki;
            cidx[i] = ij; cidx[j] = ii;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < k; i += 1024) {
    const int idx = cidx[i];
    out_idx[(int64_t)blockIdx.x * k + i] = idx;
    out_val[(int64_t)blockIdx.x * k + i] = row[idx];
  }
}

}  // namespace

extern "C" {

int omnia_mean_pool_l2(float* out, const void* hidden, int64_t stride, const int* cu, int B,
                       int D, hipStream_t s) {
  if (D % 8 || D > 8192) return -1;
  if (B == 0) return 0;
  const int vec = (D + 2047) / 2048;
#define OMNIA_POOL(V) \
  mean_pool_l2_kernel<V><<<B, 256, 0, s>>>(out, (const bf16_t*)hidden, stride, cu, D)
  if (vec <= 1) OMNIA_POOL(1);
  else if (vec <= 2) OMNIA_POOL(2);
  else OMNIA_POOL(4);
#undef OMNIA_POOL
  return (int)hipGetLastError();
}

int omnia_cosine_scores(float* scores, const float* q, int nq, const void* m, int64_t N, int D,
                        const uint8_t* valid, hipStream_t s) {
  if (D % 8) return -1;
  if ((int64_t)nq * D * 4 > 64 * 1024) return -2;
  if (N == 0) return 0;
  int64_t blocks = (N + 31) / 32;
  if (blocks > 8192) blocks = 8192;
  const size_t lds = (size_t)nq * D * 4;
#define OMNIA_COS(NQ_)                                                                   \
  cosine_scores_kernel<NQ_><<<(int)blocks, 256, lds, s>>>(scores, q, (const bf16_t*)m, N, \
                                                          D, valid)
  switch (nq) {
    case 1: OMNIA_COS(1); break;
    case 2: OMNIA_COS(2); break;
    case 4: OMNIA_COS(4); break;
    case 8: OMNIA_COS(8); break;
    default: return -3;
  }
#undef OMNIA_COS
  return (int)hipGetLastError();
}

int omnia_topk(int* out_idx, float* out_val, const float* scores, int nq, int64_t N, int k,
               hipStream_t s) {
  if (k <= 0 || k > 1024 || k > N) return -1;
  if (N > 2147483647LL) return -2;
  topk_kernel<<<nq, 1024, 0, s>>>(out_idx, out_val, scores, N, k);
  return (int)hipGetLastError();
}

}  // extern "C"
