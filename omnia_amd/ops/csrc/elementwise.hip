// Memory-bound fused ops for the Llama-family forward on gfx950:
//   * RMSNorm and fused residual-add + RMSNorm          
//   * RoPE (neox half-rotation) fused with the paged KV-cache write (K4 + K5)
//   * SwiGLU activation  silu(g) * u                     (K9 epilogue)
//   * token-embedding gather                             (K1)
// All loads/stores are 16 B per lane (8 x bf16), the HBM sweet spot on CDNA4.
#include "common.h"

using namespace omnia;

namespace {

// ---------------------------------------------------------------- RMSNorm
// One workgroup per row.  VEC = 16-byte chunks held per thread (d <= 256*8*VEC).
template <int VEC, bool ADD>
__global__ __launch_bounds__(256) void rmsnorm_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ x, bf16_t* __restrict__ residual,
    const bf16_t* __restrict__ w, int d, int64_t x_stride, int64_t out_stride, float eps) {
  __shared__ float scratch[8];
  const int row = blockIdx.x;
  const bf16_t* xr = x + (int64_t)row * x_stride;
  bf16_t* rr = ADD ? residual + (int64_t)row * d : nullptr;
  short8 v[VEC], r[VEC], wv[VEC];
  // all global loads first (x, residual, weight are independent): one memory
  // round trip before the reduction instead of three
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    const int c = (i * 256 + threadIdx.x) * 8;
    if (c < d) {
      v[i] = *reinterpret_cast<const short8*>(xr + c);
      if (ADD) r[i] = *reinterpret_cast<const short8*>(rr + c);
      wv[i] = *reinterpret_cast<const short8*>(w + c);
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    const int c = (i * 256 + threadIdx.x) * 8;
    if (c < d) {
      if (ADD) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          v[i][j] = (short)f2bf(bf2f((uint16_t)v[i][j]) + bf2f((uint16_t)r[i][j]));
        *reinterpret_cast<short8*>(rr + c) = v[i];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float f = bf2f((uint16_t)v[i][j]);
        ss += f * f;
      }
    }
  }
  ss = block_sum(ss, scratch);
  const float inv = rsqrtf(ss / (float)d + eps);
  bf16_t* orow = out + (int64_t)row * out_stride;
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    const int c = (i * 256 + threadIdx.x) * 8;
    if (c < d) {
      short8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        o[j] = (short)f2bf(bf2f((uint16_t)v[i][j]) * inv * bf2f((uint16_t)wv[i][j]));
      *reinterpret_cast<short8*>(orow + c) = o;
    }
  }
}

// ------------------------------------------------------------- RoPE + KV write
// q: [T, Hq, D] rows at q_stride; k/v: [T, Hkv, D] rows at kv_stride (views into
// the fused QKV GEMM output).  cos_sin: [max_pos, D] fp32 = (cos[D/2] | sin[D/2]).
// Cache layout: [num_blocks, Hkv, BS, D] (token rows of one head contiguous in a
// page, so decode streams 256-B rows back to back).
// One workgroup per token; each thread rotates 4 pairs (8-byte loads).
__global__ __launch_bounds__(256) void rope_kv_kernel(
    bf16_t* __restrict__ q, bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const int* __restrict__ positions, const float* __restrict__ cos_sin,
    bf16_t* __restrict__ k_cache, bf16_t* __restrict__ v_cache, const int64_t* __restrict__ slots,
    int hq, int hkv, int64_t q_stride, int64_t kv_stride, int block_size) {
  constexpr int D = 128, HALF = 64, PER = 4;  // PER pairs per thread
  const int t = blockIdx.x;
  const int pos = positions[t];
  const float* cs = cos_sin + (int64_t)pos * D;
  const int64_t slot = slots ? slots[t] : -1;
  const int units_q = hq * (HALF / PER);
  const int units_k = hkv * (HALF / PER);
  for (int u = threadIdx.x; u < units_q + units_k; u += blockDim.x) {
    const bool isq = u < units_q;
    const int uu = isq ? u : u - units_q;
    const int h = uu / (HALF / PER);
    const int i0 = (uu % (HALF / PER)) * PER;
    bf16_t* base = isq ? q + (int64_t)t * q_stride + h * D : k + (int64_t)t * kv_stride + h * D;
    short4v x1 = *reinterpret_cast<short4v*>(base + i0);
    short4v x2 = *reinterpret_cast<short4v*>(base + HALF + i0);
    short4v o1, o2;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const float c = cs[i0 + j], s = cs[HALF + i0 + j];
      const float a = bf2f((uint16_t)x1[j]), b = bf2f((uint16_t)x2[j]);
      o1[j] = (short)f2bf(a * c - b * s);
      o2[j] = (short)f2bf(b * c + a * s);
    }
    *reinterpret_cast<short4v*>(base + i0) = o1;
    *reinterpret_cast<short4v*>(base + HALF + i0) = o2;
    if (!isq && slot >= 0) {
      const int64_t blk = slot / block_size, off = slot % block_size;
      bf16_t* kc = k_cache + ((blk * hkv + h) * block_size + off) * D;
      *reinterpret_cast<short4v*>(kc + i0) = o1;
      *reinterpret_cast<short4v*>(kc + HALF + i0) = o2;
    }
  }
  if (slot >= 0) {
    // V rows: hkv * 16 chunks of 16 B
    const int64_t blk = slot / block_size, off = slot % block_size;
    for (int u = threadIdx.x; u < hkv * (D / 8); u += blockDim.x) {
      const int h = u / (D / 8), c = (u % (D / 8)) * 8;
      short8 vv = *reinterpret_cast<const short8*>(v + (int64_t)t * kv_stride + h * D + c);
      *reinterpret_cast<short8*>(v_cache + ((blk * hkv + h) * block_size + off) * D + c) = vv;
    }
  }
}

// --------------------------------------------------------------- SwiGLU
// x: [T, 2*I] (gate | up), out: [T, I].  grid (ceil(I/8/256), T): one token row per
// blockIdx.y, so no 64-bit division in the index math.
__global__ __launch_bounds__(256) void silu_mul_kernel(bf16_t* __restrict__ out,
                                                       const bf16_t* __restrict__ x,
                                                       int inter) {
  const int t = blockIdx.y;
  const int c = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= inter) return;
  const bf16_t* row = x + (int64_t)t * 2 * inter;
  const short8 g = *reinterpret_cast<const short8*>(row + c);
  const short8 u = *reinterpret_cast<const short8*>(row + inter + c);
  short8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float gf = bf2f((uint16_t)g[j]);
    const float sg = gf * __builtin_amdgcn_rcpf(1.f + __expf(-gf));
    o[j] = (short)f2bf(sg * bf2f((uint16_t)u[j]));
  }
  *reinterpret_cast<short8*>(out + (int64_t)t * inter + c) = o;
}

// --------------------------------------------------------------- embedding
// src (optional): decode rows whose input token is still on the device -- the
// token sampled by an earlier step sits in tok_slots[src[t]] when src[t] >= 0
// (async scheduling), else ids[t] holds it; resolving it here keeps the
// captured decode graph free of gather / select framework ops
__global__ __launch_bounds__(256) void embedding_kernel(bf16_t* __restrict__ out,
                                                        const int* __restrict__ ids,
                                                        const bf16_t* __restrict__ w, int d,
                                                        int vocab_start, int vocab_end,
                                                        const int64_t* __restrict__ src,
                                                        const int* __restrict__ tok_slots) {
  const int t = blockIdx.x;
  const int64_t sl = src ? src[t] : -1;
  const int id = sl >= 0 ? tok_slots[sl] : ids[t];
  const bool local = id >= vocab_start && id < vocab_end;
  const bf16_t* wr = w + (int64_t)(local ? id - vocab_start : 0) * d;
  for (int c = threadIdx.x * 8; c < d; c += blockDim.x * 8) {
    short8 v = local ? *reinterpret_cast<const short8*>(wr + c) : short8{0, 0, 0, 0, 0, 0, 0, 0};
    *reinterpret_cast<short8*>(out + (int64_t)t * d + c) = v;
  }
}

}  // namespace

extern "C" {

int omnia_rmsnorm(void* out, const void* x, void* residual, const void* w, int rows, int d,
                  int64_t x_stride, int64_t out_stride, float eps, hipStream_t s) {
  if (d % 8) return -1;
  const int vec = (d + 2047) / 2048;
  dim3 grid(rows), block(256);
#define OMNIA_NORM(V)                                                                         \
  if (residual)                                                                               \
    rmsnorm_kernel<V, true><<<grid, block, 0, s>>>((bf16_t*)out, (const bf16_t*)x,            \
                                                   (bf16_t*)residual, (const bf16_t*)w, d,    \
                                                   x_stride, out_stride, eps);                \
  else                                                                                        \
    rmsnorm_kernel<V, false><<<grid, block, 0, s>>>((bf16_t*)out, (const bf16_t*)x, nullptr,  \
                                                    (const bf16_t*)w, d, x_stride, out_stride, \
                                                    eps);
  if (vec <= 1) { OMNIA_NORM(1) }
  else if (vec <= 2) { OMNIA_NORM(2) }
  else if (vec <= 4) { OMNIA_NORM(4) }
  else if (vec <= 8) { OMNIA_NORM(8) }
  else return -2;
#undef OMNIA_NORM
  return (int)hipGetLastError();
}

int omnia_rope_kv(void* q, void* k, const void* v, const int* positions, const float* cos_sin,
                  void* k_cache, void* v_cache, const int64_t* slots, int T, int hq, int hkv,
                  int head_dim, int64_t q_stride, int64_t kv_stride, int block_size,
                  hipStream_t s) {
  if (head_dim != 128) return -1;
  if (T == 0) return 0;
  rope_kv_kernel<<<T, 256, 0, s>>>((bf16_t*)q, (bf16_t*)k, (const bf16_t*)v, positions, cos_sin,
                                   (bf16_t*)k_cache, (bf16_t*)v_cache, slots, hq, hkv, q_stride,
                                   kv_stride, block_size);
  return (int)hipGetLastError();
}

int omnia_silu_mul(void* out, const void* x, int64_t T, int inter, hipStream_t s) {
  if (inter % 8) return -1;
  if (T == 0) return 0;
  if (T > 2147483647LL) return -2;
  dim3 grid((inter / 8 + 255) / 256, (unsigned)T);
  silu_mul_kernel<<<grid, 256, 0, s>>>((bf16_t*)out, (const bf16_t*)x, inter);
  return (int)hipGetLastError();
}

int omnia_embedding(void* out, const int* ids, const void* w, int T, int d, int vocab_start,
                    int vocab_end, const int64_t* src, const int* tok_slots, hipStream_t s) {
  if (d % 8) return -1;
  if (src && !tok_slots) return -2;
  if (T == 0) return 0;
  embedding_kernel<<<T, 256, 0, s>>>((bf16_t*)out, ids, (const bf16_t*)w, d, vocab_start,
                                     vocab_end, src, tok_slots);
  return (int)hipGetLastError();
}

}  // extern "C"
