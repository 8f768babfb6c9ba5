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
// Partial loads are 16 B per lane (4 floats); S <= 16.
#include "common.h"

using namespace omnia;

namespace {

// sum over the S slabs of 4 consecutive floats at element offset e
__device__ __forceinline__ float4v sum4(const float* __restrict__ p, int S, int64_t slab,
                                        int64_t e) {
  float4v a = *reinterpret_cast<const float4v*>(p + e);
  for (int s = 1; s < S; ++s) a += *reinterpret_cast<const float4v*>(p + s * slab + e);
  return a;
}

__device__ __forceinline__ float rnd(float x) { return bf2f(f2bf(x)); }  // bf16 rounding

// ------------------------------------------------------ residual add + RMSNorm
// one workgroup (256 threads) per row; VEC chunks of 8 columns per thread
template <int VEC>
__global__ __launch_bounds__(256) void splitk_add_rmsnorm_kernel(
    bf16_t* __restrict__ out, const float* __restrict__ parts, bf16_t* __restrict__ residual,
    const bf16_t* __restrict__ w, int S, int M, int d, float eps) {
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
      const float4v a = sum4(parts, S, slab, e), b = sum4(parts, S, slab, e + 4);
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
// parts [S][T][(hq + 2 hkv) * D]; one workgroup per token; a thread rotates 4
// pairs (q or k) or copies 8 v elements.  Same cache layout as rope_kv_kernel:
// [num_blocks, Hkv, BS, D].
__global__ __launch_bounds__(256) void splitk_rope_kv_kernel(
    bf16_t* __restrict__ q, const float* __restrict__ parts, int S, int T,
    const int* __restrict__ positions, const float* __restrict__ cos_sin,
    bf16_t* __restrict__ k_cache, bf16_t* __restrict__ v_cache, const int64_t* __restrict__ slots,
    int hq, int hkv, int block_size) {
  constexpr int D = 128, HALF = 64, PER = 4;
  const int t = blockIdx.x;
  const int N = (hq + 2 * hkv) * D;
  const int64_t slab = (int64_t)T * N;
  const float* row = parts + (int64_t)t * N;
  const int pos = positions[t];
  const float* cs = cos_sin + (int64_t)pos * D;
  const int64_t slot = slots[t];
  const int64_t blk = slot >= 0 ? slot / block_size : 0, off = slot >= 0 ? slot % block_size : 0;
  const int units_q = hq * (HALF / PER), units_k = hkv * (HALF / PER);
  for (int u = threadIdx.x; u < units_q + units_k; u += blockDim.x) {
    const bool isq = u < units_q;
    const int uu = isq ? u : u - units_q;
    const int h = uu / (HALF / PER);
    const int i0 = (uu % (HALF / PER)) * PER;
    const int64_t base = isq ? (int64_t)h * D : (int64_t)(hq + h) * D;
    const float4v x1 = sum4(row, S, slab, base + i0), x2 = sum4(row, S, slab, base + HALF + i0);
    short4v o1, o2;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const float c = cs[i0 + j], s = cs[HALF + i0 + j];
      const float a = rnd(x1[j]), b = rnd(x2[j]);  // bf16 projection output, as unfused
      o1[j] = (short)f2bf(a * c - b * s);
      o2[j] = (short)f2bf(b * c + a * s);
    }
    if (isq) {
      bf16_t* qr = q + (int64_t)t * hq * D + h * D;
      *reinterpret_cast<short4v*>(qr + i0) = o1;
      *reinterpret_cast<short4v*>(qr + HALF + i0) = o2;
    } else if (slot >= 0) {
      bf16_t* kc = k_cache + ((blk * hkv + h) * block_size + off) * D;
      *reinterpret_cast<short4v*>(kc + i0) = o1;
      *reinterpret_cast<short4v*>(kc + HALF + i0) = o2;
    }
  }
  if (slot >= 0) {
    for (int u = threadIdx.x; u < hkv * (D / 8); u += blockDim.x) {
      const int h = u / (D / 8), c = (u % (D / 8)) * 8;
      const int64_t e = (int64_t)(hq + hkv + h) * D + c;
      const float4v a = sum4(row, S, slab, e), b = sum4(row, S, slab, e + 4);
      short8 vv;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        vv[j] = (short)f2bf(a[j]);
        vv[j + 4] = (short)f2bf(b[j]);
      }
      *reinterpret_cast<short8*>(v_cache + ((blk * hkv + h) * block_size + off) * D + c) = vv;
    }
  }
}

// --------------------------------------------------------------- SwiGLU
// parts [S][M][2I] (gate | up) -> out [M, I]; grid (ceil(I/8/256), M)
__global__ __launch_bounds__(256) void splitk_swiglu_kernel(bf16_t* __restrict__ out,
                                                            const float* __restrict__ parts,
                                                            int S, int M, int inter) {
  const int m = blockIdx.y;
  const int c = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= inter) return;
  const int64_t slab = (int64_t)M * 2 * inter;
  const int64_t e = (int64_t)m * 2 * inter + c;
  const float4v g0 = sum4(parts, S, slab, e), g1 = sum4(parts, S, slab, e + 4);
  const float4v u0 = sum4(parts, S, slab, e + inter), u1 = sum4(parts, S, slab, e + inter + 4);
  short8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float g = rnd(j < 4 ? g0[j] : g1[j - 4]), u = rnd(j < 4 ? u0[j] : u1[j - 4]);
    o[j] = (short)f2bf(g * __builtin_amdgcn_rcpf(1.f + __expf(-g)) * u);
  }
  *reinterpret_cast<short8*>(out + (int64_t)m * inter + c) = o;
}

// --------------------------------------------------------------- reduce
__global__ __launch_bounds__(256) void splitk_reduce_kernel(bf16_t* __restrict__ out,
                                                            const float* __restrict__ parts,
                                                            int S, int64_t n) {
  const int64_t e = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (e >= n) return;
  const float4v a = sum4(parts, S, n, e), b = sum4(parts, S, n, e + 4);
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

int omnia_splitk_add_rmsnorm(void* out, const float* parts, void* residual, const void* w, int S,
                             int M, int d, float eps, hipStream_t s) {
  if (S < 1 || S > 16 || d % 8 || M < 1) return -1;
  const int vec = (d + 2047) / 2048;
#define OMNIA_SKN(V)                                                                            \
  splitk_add_rmsnorm_kernel<V><<<M, 256, 0, s>>>((bf16_t*)out, parts, (bf16_t*)residual,        \
                                                 (const bf16_t*)w, S, M, d, eps);
  if (vec <= 1) { OMNIA_SKN(1) }
  else if (vec <= 2) { OMNIA_SKN(2) }
  else if (vec <= 4) { OMNIA_SKN(4) }
  else return -2;
#undef OMNIA_SKN
  return (int)hipGetLastError();
}

int omnia_splitk_rope_kv(void* q, const float* parts, int S, int T, const int* positions,
                         const float* cos_sin, void* k_cache, void* v_cache, const int64_t* slots,
                         int hq, int hkv, int head_dim, int block_size, hipStream_t s) {
  if (head_dim != 128 || S < 1 || S > 16) return -1;
  if (T == 0) return 0;
  splitk_rope_kv_kernel<<<T, 256, 0, s>>>((bf16_t*)q, parts, S, T, positions, cos_sin,
                                          (bf16_t*)k_cache, (bf16_t*)v_cache, slots, hq, hkv,
                                          block_size);
  return (int)hipGetLastError();
}

int omnia_splitk_swiglu(void* out, const float* parts, int S, int M, int inter, hipStream_t s) {
  if (S < 1 || S > 16 || inter % 8 || M < 1) return -1;
  dim3 grid((inter / 8 + 255) / 256, M);
  splitk_swiglu_kernel<<<grid, 256, 0, s>>>((bf16_t*)out, parts, S, M, inter);
  return (int)hipGetLastError();
}

int omnia_splitk_reduce(void* out, const float* parts, int S, int64_t n, hipStream_t s) {
  if (S < 1 || S > 16 || n % 8) return -1;
  if (n == 0) return 0;
  splitk_reduce_kernel<<<(unsigned)((n / 8 + 255) / 256), 256, 0, s>>>((bf16_t*)out, parts, S,
                                                                       n);
  return (int)hipGetLastError();
}

}  // extern "C"
