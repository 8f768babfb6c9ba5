// Split-K consumers: the kernels that follow a decode projection reduce the
// projection's S fp32 partial slabs (wgemm.hip MODE 2, [S][M][N]) as part of
// their own work, so split-K needs no combine launch and the projection's
// output never exists in bf16 (QKV + RoPE + KV write,
// O / down + residual + RMSNorm).
//   splitk_rope_kv      QKV partials -> RoPE(q) bf16 [T, Hq*D], RoPE(k) and v
//                       written straight into the paged KV cache
//   splitk_add_rmsnorm  residual += bf16(sum); out = RMSNorm(residual) * w
//   splitk_swiglu       gate_up partials -> silu(g) * u bf16 [M, I]
//   splitk_reduce       bf16(sum) [M, N] (TP: before the all-reduce)
// Partial loads are 16 B per lane (4 floats); S <= 16.  Every kernel is
// instantiated per slab count S: with a compile-time S the S loads of a sum are
// issued back to back (with a runtime trip count hipcc waited for each load
// before issuing the next, serialising S memory latencies per element).
#include "common.h"

using namespace omnia;

namespace {

// sum over the S slabs of 4 consecutive floats at element offset e
// Slabs are fp32 or fp16 (tgemm MODE 3: half the slab bytes for the producer
// and the consumer; each fp16 slab holds one K-slice's fp32 sum rounded to 11
// bits, below the bf16 rounding of the projection's output)
typedef _Float16 half4v __attribute__((ext_vector_type(4)));

template <typename P>
__device__ __forceinline__ float4v load4(const P* __restrict__ p) {
  if constexpr (sizeof(P) == 4) {
    return *reinterpret_cast<const float4v*>(p);
  } else {
    const half4v h = *reinterpret_cast<const half4v*>(p);
    return float4v{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
  }
}

template <int S, typename P>
__device__ __forceinline__ float4v sum4(const P* __restrict__ p, int64_t slab, int64_t e) {
  float4v v[S];
#pragma unroll
  for (int s = 0; s < S; ++s) v[s] = load4(p + s * slab + e);
  float4v a = v[0];
#pragma unroll
  for (int s = 1; s < S; ++s) a += v[s];
  return a;
}

#define OMNIA_SPLITK_S(X) \
  X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16)

__device__ __forceinline__ float rnd(float x) { return bf2f(f2bf(x)); }  // bf16 rounding

// ------------------------------------------------------ residual add + RMSNorm
// one workgroup (256 threads) per row; VEC chunks of 8 columns per thread
template <int VEC, int S, typename P>
__global__ __launch_bounds__(256) void splitk_add_rmsnorm_kernel(
    bf16_t* __restrict__ out, const P* __restrict__ parts, bf16_t* __restrict__ residual,
    const bf16_t* __restrict__ w, int M, int d, float eps) {
  __shared__ float scratch[8];
  const int row = blockIdx.x;
  const int64_t slab = (int64_t)M * d;
  float v[VEC][8];
  short8 wv[VEC];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    const int c = (i * 256 + threadIdx.x) * 8;
    if (c < d) {
      const int64_t e = (int64_t)row * d + c;
      const float4v a = sum4<S>(parts, slab, e), b = sum4<S>(parts, slab, e + 4);
      const short8 r = *reinterpret_cast<const short8*>(residual + e);
      wv[i] = *reinterpret_cast<const short8*>(w + c);
      short8 nr;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = rnd(j < 4 ? a[j] : b[j - 4]);  // the projection's bf16 output
        const float y = rnd(x + bf2f((uint16_t)r[j]));
        v[i][j] = y;
        nr[j] = (short)f2bf(y);
        ss += y * y;
      }
      *reinterpret_cast<short8*>(residual + e) = nr;
    }
  }
  ss = block_sum(ss, scratch);
  const float inv = rsqrtf(ss / (float)d + eps);
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    const int c = (i * 256 + threadIdx.x) * 8;
    if (c < d) {
      short8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (short)f2bf(v[i][j] * inv * bf2f((uint16_t)wv[i][j]));
      *reinterpret_cast<short8*>(out + (int64_t)row * d + c) = o;
    }
  }
}

// ------------------------------------------------------------- RoPE + KV write
// parts [S][T][(hq + 2 hkv) * D]; grid (T, ceil((hq + 2 hkv) / 16)): a block
// covers 16 heads of one token, 16 threads per head, ONE unit per thread -- 4
// rotation pairs of a q or k head, or 8 elements of a v head -- so every slab
// load of the block is in flight at once.  Same cache layout as rope_kv_kernel:
// [num_blocks, Hkv, BS, D].
template <int S, typename P>
__global__ __launch_bounds__(256) void splitk_rope_kv_kernel(
    bf16_t* __restrict__ q, const P* __restrict__ parts, int T,
    const int* __restrict__ positions, const float* __restrict__ cos_sin,
    bf16_t* __restrict__ k_cache, bf16_t* __restrict__ v_cache, const int64_t* __restrict__ slots,
    int hq, int hkv, int block_size) {
  constexpr int D = 128, HALF = 64, PER = 4;
  const int t = blockIdx.x;
  const int head = blockIdx.y * 16 + (threadIdx.x >> 4), sub = threadIdx.x & 15;
  if (head >= hq + 2 * hkv) return;
  const int N = (hq + 2 * hkv) * D;
  const int64_t slab = (int64_t)T * N;
  const P* row = parts + (int64_t)t * N;
  const int64_t slot = slots[t];
  const int64_t blk = slot >= 0 ? slot / block_size : 0, off = slot >= 0 ? slot % block_size : 0;
  if (head >= hq + hkv) {  // v: 8 contiguous elements straight into the cache
    if (slot < 0) return;
    const int h = head - hq - hkv, c = sub * 8;
    const int64_t e = (int64_t)head * D + c;
    const float4v a = sum4<S>(row, slab, e), b = sum4<S>(row, slab, e + 4);
    short8 vv;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      vv[j] = (short)f2bf(a[j]);
      vv[j + 4] = (short)f2bf(b[j]);
    }
    *reinterpret_cast<short8*>(v_cache + ((blk * hkv + h) * block_size + off) * D + c) = vv;
    return;
  }
  const bool isq = head < hq;
  if (!isq && slot < 0) return;
  const int i0 = sub * PER;
  const int64_t base = (int64_t)head * D;
  const float4v x1 = sum4<S>(row, slab, base + i0), x2 = sum4<S>(row, slab, base + HALF + i0);
  const float* cs = cos_sin + (int64_t)positions[t] * D;
  short4v o1, o2;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const float c = cs[i0 + j], s = cs[HALF + i0 + j];
    const float a = rnd(x1[j]), b = rnd(x2[j]);  // bf16 projection output, as unfused
    o1[j] = (short)f2bf(a * c - b * s);
    o2[j] = (short)f2bf(b * c + a * s);
  }
  bf16_t* dst = isq ? q + (int64_t)t * hq * D + head * D
                    : k_cache + ((blk * hkv + (head - hq)) * block_size + off) * D;
  *reinterpret_cast<short4v*>(dst + i0) = o1;
  *reinterpret_cast<short4v*>(dst + HALF + i0) = o2;
}

// --------------------------------------------------------------- SwiGLU
// parts [S][M][2I] (gate | up) -> out [M, I]; grid (ceil(I/8/256), M)
template <int S, typename P>
__global__ __launch_bounds__(256) void splitk_swiglu_kernel(bf16_t* __restrict__ out,
                                                            const P* __restrict__ parts,
                                                            int M, int inter) {
  const int m = blockIdx.y;
  const int c = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= inter) return;
  const int64_t slab = (int64_t)M * 2 * inter;
  const int64_t e = (int64_t)m * 2 * inter + c;
  const float4v g0 = sum4<S>(parts, slab, e), g1 = sum4<S>(parts, slab, e + 4);
  const float4v u0 = sum4<S>(parts, slab, e + inter), u1 = sum4<S>(parts, slab, e + inter + 4);
  short8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float g = rnd(j < 4 ? g0[j] : g1[j - 4]), u = rnd(j < 4 ? u0[j] : u1[j - 4]);
    o[j] = (short)f2bf(g * __builtin_amdgcn_rcpf(1.f + __expf(-g)) * u);
  }
  *reinterpret_cast<short8*>(out + (int64_t)m * inter + c) = o;
}

// --------------------------------------------------------------- reduce
template <int S, typename P>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(bf16_t* __restrict__ out,
                                                            const P* __restrict__ parts,
                                                            int64_t n) {
  const int64_t e = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (e >= n) return;
  const float4v a = sum4<S>(parts, n, e), b = sum4<S>(parts, n, e + 4);
  short8 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[j] = (short)f2bf(a[j]);
    o[j + 4] = (short)f2bf(b[j]);
  }
  *reinterpret_cast<short8*>(out + e) = o;
}

}  // namespace

extern "C" {

int omnia_splitk_add_rmsnorm(void* out, const void* parts, int half, void* residual,
                             const void* w, int S, int M, int d, float eps, hipStream_t st) {
  if (S < 1 || S > 16 || d % 8 || M < 1) return -1;
  const int vec = (d + 2047) / 2048;
  if (vec > 4) return -2;
#define OMNIA_SKN(V, SS)                                                                       \
  if (half)                                                                                    \
    splitk_add_rmsnorm_kernel<V, SS, _Float16><<<M, 256, 0, st>>>(                             \
        (bf16_t*)out, (const _Float16*)parts, (bf16_t*)residual, (const bf16_t*)w, M, d, eps);  \
  else                                                                                         \
    splitk_add_rmsnorm_kernel<V, SS, float><<<M, 256, 0, st>>>(                                \
        (bf16_t*)out, (const float*)parts, (bf16_t*)residual, (const bf16_t*)w, M, d, eps);
#define OMNIA_SKS(SS)                              \
  if (S == SS) {                                   \
    if (vec <= 1) { OMNIA_SKN(1, SS) }             \
    else if (vec <= 2) { OMNIA_SKN(2, SS) }        \
    else { OMNIA_SKN(4, SS) }                      \
  }
  OMNIA_SPLITK_S(OMNIA_SKS)
#undef OMNIA_SKS
#undef OMNIA_SKN
  return (int)hipGetLastError();
}

int omnia_splitk_rope_kv(void* q, const void* parts, int half, int S, int T, const int* positions,
                         const float* cos_sin, void* k_cache, void* v_cache, const int64_t* slots,
                         int hq, int hkv, int head_dim, int block_size, hipStream_t s) {
  if (head_dim != 128 || S < 1 || S > 16) return -1;
  if (T == 0) return 0;
  const dim3 grid(T, (hq + 2 * hkv + 15) / 16);
#define OMNIA_SKR(SS)                                                                          \
  if (S == SS) {                                                                               \
    if (half)                                                                                  \
      splitk_rope_kv_kernel<SS, _Float16><<<grid, 256, 0, s>>>(                                \
          (bf16_t*)q, (const _Float16*)parts, T, positions, cos_sin, (bf16_t*)k_cache,         \
          (bf16_t*)v_cache, slots, hq, hkv, block_size);                                       \
    else                                                                                       \
      splitk_rope_kv_kernel<SS, float><<<grid, 256, 0, s>>>(                                   \
          (bf16_t*)q, (const float*)parts, T, positions, cos_sin, (bf16_t*)k_cache,            \
          (bf16_t*)v_cache, slots, hq, hkv, block_size);                                       \
  }
  OMNIA_SPLITK_S(OMNIA_SKR)
#undef OMNIA_SKR
  return (int)hipGetLastError();
}

int omnia_splitk_swiglu(void* out, const void* parts, int half, int S, int M, int inter,
                        hipStream_t s) {
  if (S < 1 || S > 16 || inter % 8 || M < 1) return -1;
  dim3 grid((inter / 8 + 255) / 256, M);
#define OMNIA_SKW(SS)                                                                          \
  if (S == SS) {                                                                               \
    if (half)                                                                                  \
      splitk_swiglu_kernel<SS, _Float16><<<grid, 256, 0, s>>>((bf16_t*)out,                    \
                                                             (const _Float16*)parts, M, inter); \
    else                                                                                       \
      splitk_swiglu_kernel<SS, float><<<grid, 256, 0, s>>>((bf16_t*)out, (const float*)parts,  \
                                                          M, inter);                           \
  }
  OMNIA_SPLITK_S(OMNIA_SKW)
#undef OMNIA_SKW
  return (int)hipGetLastError();
}

int omnia_splitk_reduce(void* out, const void* parts, int half, int S, int64_t n, hipStream_t s) {
  if (S < 1 || S > 16 || n % 8) return -1;
  if (n == 0) return 0;
  const unsigned g = (unsigned)((n / 8 + 255) / 256);
#define OMNIA_SKD(SS)                                                                          \
  if (S == SS) {                                                                               \
    if (half)                                                                                  \
      splitk_reduce_kernel<SS, _Float16><<<g, 256, 0, s>>>((bf16_t*)out, (const _Float16*)parts, \
                                                           n);                                 \
    else                                                                                       \
      splitk_reduce_kernel<SS, float><<<g, 256, 0, s>>>((bf16_t*)out, (const float*)parts, n); \
  }
  OMNIA_SPLITK_S(OMNIA_SKD)
#undef OMNIA_SKD
  return (int)hipGetLastError();
}

}  // extern "C"
