// Mixture-of-Experts kernels for gfx950:
//   * moe_topk   : router softmax + top-k (+ renormalise over the selected
//                  experts, Mixtral semantics); one wave per token, E <= 64
//   * moe_align  : per-expert counts -> 64-row-padded offsets -> token
//                  permutation (sorted assignment ids) + block->expert map, all on
//                  device, so the grouped GEMM grid never needs a host sync
//                  (graph-capturable decode)
//   * moe_gemm   : grouped MFMA GEMM over the expert-sorted rows.
//                  MODE 0: gate_up with the SwiGLU epilogue fused (a 64-column
//                          tile = 32 gate + the matching 32 up columns)
//                  MODE 1: down projection with the routing weight fused, rows
//                          written back to their (token, slot) position
//   * moe_combine: out[t] = sum_j Y[t*k + j]  (deterministic, no atomics)
// Expert parallelism: moe_align keeps only experts in [e_lo, e_hi); the caller
// all-reduces the combined output over the EP group.
#include "common.h"

using namespace omnia;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float4v mfma16(short8 a, short8 b, float4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

constexpr int BM = 64;  // rows per grouped-GEMM block (and alignment of expert segments)

// ------------------------------------------------------------------ top-k
template <typename T>
__device__ __forceinline__ float ld(const T* p);
template <>
__device__ __forceinline__ float ld<float>(const float* p) { return *p; }
template <>
__device__ __forceinline__ float ld<bf16_t>(const bf16_t* p) { return bf2f(*p); }

// one wave per token: lane e (< E) holds expert e's logit x; writes the token's
// k (id, weight) pairs -- softmax over all E, top-k, optional renormalisation
__device__ __forceinline__ void select_topk(float x, int lane, int t, int E, int k, int renorm,
                                            int* __restrict__ ids, float* __restrict__ wts) {
  if (!(x == x)) x = -INFINITY;  // NaN logits (e.g. a padded row) never win a slot
  const float m = wave_max(x);
  // an all -inf row (padding) routes uniformly instead of producing NaN weights
  const bool flat = !(m > -INFINITY);
  const float p = lane < E ? (flat ? 1.f : __expf(x - m)) : 0.f;
  const float total = wave_sum(p);
  bool taken = false;
  int my_slot = -1;
  float sel = 0.f, mine = 0.f;
  for (int j = 0; j < k; ++j) {
    const float v = taken ? -INFINITY : x;
    const float vm = wave_max(v);
    // only untaken experts compete, so every slot gets a distinct valid id in [0, E)
    const uint64_t b = __ballot(!taken && v == vm && lane < E);
    const int first = __ffsll((unsigned long long)b) - 1;  // lowest index wins ties
    const float pj = flat ? 1.f : __expf(vm - m);
    if (lane == first) {
      taken = true;
      my_slot = j;
      mine = pj;
    }
    sel += pj;
    if (lane == 0) ids[(int64_t)t * k + j] = first;
  }
  const float denom = renorm ? sel : total;
  if (taken) wts[(int64_t)t * k + my_slot] = mine / denom;
}

template <typename T>
__global__ __launch_bounds__(256) void moe_topk_kernel(int* __restrict__ ids,
                                                       float* __restrict__ wts,
                                                       const T* __restrict__ logits, int n_tok,
                                                       int E, int k, int renorm) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= n_tok) return;
  const float x = lane < E ? ld<T>(logits + (int64_t)t * E + lane) : -INFINITY;
  select_topk(x, lane, t, E, k, renorm, ids, wts);
}

// Router GEMM fused with the top-k: logits[t][e] = x[t] . router[e] computed
// by the token's wave (lane = 8-element chunks of d; the E router rows are a few
// KB per expert and stay L2-resident), rounded to bf16 as a bf16 linear layer
// would produce them, then selected in-wave -- no [T, E] logits tensor and no
// library GEMM on the MoE path.
template <int E_MAX>
__global__ __launch_bounds__(256) void moe_router_topk_kernel(
    int* __restrict__ ids, float* __restrict__ wts, const bf16_t* __restrict__ x,
    const bf16_t* __restrict__ router, int n_tok, int d, int E, int k, int renorm) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= n_tok) return;
  const bf16_t* xr = x + (int64_t)t * d;
  float acc[E_MAX];
#pragma unroll
  for (int e = 0; e < E_MAX; ++e) acc[e] = 0.f;
  for (int c = lane * 8; c < d; c += 64 * 8) {
    const short8 xv = *reinterpret_cast<const short8*>(xr + c);
    float xf[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) xf[j] = bf2f((uint16_t)xv[j]);
#pragma unroll
    for (int e = 0; e < E_MAX; ++e) {
      if (e < E) {
        const short8 wv = *reinterpret_cast<const short8*>(router + (int64_t)e * d + c);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[e] += xf[j] * bf2f((uint16_t)wv[j]);
      }
    }
  }
  float mine = -INFINITY;
#pragma unroll
  for (int e = 0; e < E_MAX; ++e) {
    if (e < E) {
      const float v = bf2f(f2bf(wave_sum(acc[e])));
      if (lane == e) mine = v;
    }
  }
  select_topk(mine, lane, t, E, k, renorm, ids, wts);
}

// ------------------------------------------------------------------ align
// One 1024-thread workgroup.  n = T*k assignments.  sorted has max_blocks*BM
// entries (n = padding sentinel), blk_expert max_blocks entries.
// bm: the segment alignment = the grouped GEMM's row tile (64 here, 256 for the
// 256x256 prefill tile of pgemm.hip EPI 5 / 6)
__global__ __launch_bounds__(1024) void moe_align_kernel(int* __restrict__ sorted,
                                                         int* __restrict__ blk_expert,
                                                         int* __restrict__ n_blocks,
                                                         const int* __restrict__ ids, int n,
                                                         int E, int e_lo, int e_hi,
                                                         int max_blocks, int bm) {
  __shared__ int cnt[256];
  __shared__ int off[257];
  __shared__ int cur[256];
  const int tid = threadIdx.x;
  for (int e = tid; e < E; e += 1024) cnt[e] = 0;
  for (int r = tid; r < max_blocks * bm; r += 1024) sorted[r] = n;
  for (int b = tid; b < max_blocks; b += 1024) blk_expert[b] = -1;
  __syncthreads();
  for (int i = tid; i < n; i += 1024) {
    const int e = ids[i];
    if (e >= e_lo && e < e_hi) atomicAdd(&cnt[e], 1);
  }
  __syncthreads();
  if (tid == 0) {
    off[0] = 0;
    for (int e = 0; e < E; ++e) off[e + 1] = off[e] + (cnt[e] + bm - 1) / bm * bm;
    *n_blocks = off[E] / bm;
  }
  __syncthreads();
  for (int e = tid; e < E; e += 1024) cur[e] = off[e];
  for (int b = tid; b < off[E] / bm; b += 1024) {
    int e = 0;
    while (off[e + 1] <= b * bm) ++e;
    blk_expert[b] = e;
  }
  __syncthreads();
  for (int i = tid; i < n; i += 1024) {
    const int e = ids[i];
    if (e >= e_lo && e < e_hi) sorted[atomicAdd(&cur[e], 1)] = i;
  }
}

// ------------------------------------------------------------------ grouped GEMM
// LDS image: [64 rows][8 chunks of 16 B], chunk c of row r stored at c ^ (r & 7)
// (ds_read_b128 fragment reads are then conflict-free across the 16 rows).
__device__ __forceinline__ int swz(int row, int ch) { return row * 64 + ((ch ^ (row & 7)) << 3); }

template <int MODE>
__global__ __launch_bounds__(256) void moe_gemm_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
    const int* __restrict__ sorted, const int* __restrict__ blk_expert,
    const int* __restrict__ n_blocks, const float* __restrict__ route_w, int K, int N,
    int topk, int n_assign, int e_lo) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * 2 * BM * 64];
  const int mb = blockIdx.y;
  if (mb >= *n_blocks) return;
  const int e = blk_expert[mb] - e_lo;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int n0 = blockIdx.x * (MODE == 0 ? 32 : 64);
  const int w_rows = MODE == 0 ? 2 * N : N;  // rows of one expert's weight matrix
  const bf16_t* We = W + (int64_t)e * w_rows * K;

  // per-thread staging: 2 A chunks + 2 B chunks of 16 B per k-tile
  const bf16_t* a_src[2];
  const bf16_t* b_src[2];
  int a_lds[2], b_lds[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tid + i * 256;  // 0..511
    const int row = c >> 3, ch = c & 7;
    const int flat = sorted[mb * BM + row];
    const int64_t arow = MODE == 0 ? (flat < n_assign ? flat / topk : 0) : (int64_t)mb * BM + row;
    a_src[i] = A + arow * K + ch * 8;
    a_lds[i] = swz(row, ch);
    int wrow;
    if (MODE == 0)
      wrow = row < 32 ? n0 + row : N + n0 + (row - 32);
    else
      wrow = n0 + row;
    b_src[i] = We + (int64_t)wrow * K + ch * 8;
    b_lds[i] = swz(row, ch);
  }
  // Rows past the expert's assignments read row 0 of A (valid memory) and are
  // dropped in the epilogue, so every load is unconditional.  Two k-tiles of
  // loads in flight in a register ring with clamped k offsets (branch-free, so
  // hipcc counts vmcnt across the loop instead of draining it each k-step).
  auto gload = [&](short8* ra, short8* rb, int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      ra[i] = *reinterpret_cast<const short8*>(a_src[i] + k0);
      rb[i] = __builtin_nontemporal_load(reinterpret_cast<const short8*>(b_src[i] + k0));
    }
  };
  auto lstore = [&](const short8* ra, const short8* rb, int buf) {
    bf16_t* As = lds + buf * (2 * BM * 64);
    bf16_t* Bs = As + BM * 64;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      *reinterpret_cast<short8*>(As + a_lds[i]) = ra[i];
      *reinterpret_cast<short8*>(Bs + b_lds[i]) = rb[i];
    }
  };

  float4v acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = {0.f, 0.f, 0.f, 0.f};

  const int nk = K / 64;
  const int fr = lane & 15, fq = lane >> 4;
  auto compute = [&](int buf) {
    const bf16_t* As = lds + buf * (2 * BM * 64);
    const bf16_t* Bs = As + BM * 64;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const short8 a = *reinterpret_cast<const short8*>(As + swz(16 * w + fr, ks * 4 + fq));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const short8 b = *reinterpret_cast<const short8*>(Bs + swz(16 * j + fr, ks * 4 + fq));
        acc[j] = mfma16(a, b, acc[j]);
      }
    }
  };
  const int klast = (nk - 1) * 64;
  short8 ra0[2], rb0[2], ra1[2], rb1[2];
  gload(ra0, rb0, 0);
  gload(ra1, rb1, min(64, klast));
  lstore(ra0, rb0, 0);
  __syncthreads();
  for (int kt = 0; kt < nk; kt += 2) {
    gload(ra0, rb0, min((kt + 2) * 64, klast));
    compute(0);
    lstore(ra1, rb1, 1);
    __syncthreads();
    gload(ra1, rb1, min((kt + 3) * 64, klast));
    if (kt + 1 < nk) compute(1);
    lstore(ra0, rb0, 0);
    __syncthreads();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // epilogue: lane holds rows 16w + 4*fq + r, columns 16*j + fr
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = mb * BM + 16 * w + 4 * fq + r;
    const int flat = sorted[row];
    if (flat >= n_assign) continue;
    if (MODE == 0) {
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const float g = acc[jj][r], u = acc[jj + 2][r];
        const float s = g * __builtin_amdgcn_rcpf(1.f + __expf(-g));
        out[(int64_t)row * N + n0 + 16 * jj + fr] = f2bf(s * u);
      }
    } else {
      const float wt = route_w[flat];
#pragma unroll
      for (int j = 0; j < 4; ++j) out[(int64_t)flat * N + n0 + 16 * j + fr] = f2bf(wt * acc[j][r]);
    }
  }
}

// ------------------------------------------------------------------ combine
// out[t] = sum over the token's k slots whose expert is local of Y[t*k + j]
__global__ __launch_bounds__(256) void moe_combine_kernel(bf16_t* __restrict__ out,
                                                          const bf16_t* __restrict__ Y,
                                                          const int* __restrict__ ids, int d,
                                                          int topk, int e_lo, int e_hi) {
  const int t = blockIdx.x;
  for (int c = threadIdx.x * 8; c < d; c += 256 * 8) {
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < topk; ++j) {
      const int e = ids[(int64_t)t * topk + j];
      if (e < e_lo || e >= e_hi) continue;
      const short8 v = *reinterpret_cast<const short8*>(Y + ((int64_t)t * topk + j) * d + c);
#pragma unroll
      for (int q = 0; q < 8; ++q) s[q] += bf2f((uint16_t)v[q]);
    }
    short8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = (short)f2bf(s[q]);
    *reinterpret_cast<short8*>(out + (int64_t)t * d + c) = o;
  }
}

}  // namespace

extern "C" {

int omnia_moe_topk(int* ids, float* wts, const void* logits, int logits_bf16, int n_tok, int E,
                   int k, int renorm, hipStream_t s) {
  if (E > 64 || k > E || k < 1) return -1;
  if (n_tok == 0) return 0;
  const int blocks = (n_tok + 3) / 4;
  if (logits_bf16)
    moe_topk_kernel<bf16_t><<<blocks, 256, 0, s>>>(ids, wts, (const bf16_t*)logits, n_tok, E, k,
                                                   renorm);
  else
    moe_topk_kernel<float><<<blocks, 256, 0, s>>>(ids, wts, (const float*)logits, n_tok, E, k,
                                                  renorm);
  return (int)hipGetLastError();
}

int omnia_moe_router_topk(int* ids, float* wts, const void* x, const void* router, int n_tok,
                          int d, int E, int k, int renorm, hipStream_t s) {
  if (E > 64 || k > E || k < 1 || d % 8) return -1;
  if (n_tok == 0) return 0;
  const int blocks = (n_tok + 3) / 4;
#define OMNIA_RT(EM)                                                                         \
  moe_router_topk_kernel<EM><<<blocks, 256, 0, s>>>(ids, wts, (const bf16_t*)x,               \
                                                   (const bf16_t*)router, n_tok, d, E, k, renorm)
  if (E <= 8) OMNIA_RT(8);
  else if (E <= 16) OMNIA_RT(16);
  else if (E <= 32) OMNIA_RT(32);
  else OMNIA_RT(64);
#undef OMNIA_RT
  return (int)hipGetLastError();
}

int omnia_moe_max_blocks(int n_assign, int n_experts, int bm) {
  return (n_assign + n_experts * (bm - 1) + bm - 1) / bm;
}

int omnia_moe_align(int* sorted, int* blk_expert, int* n_blocks, const int* ids, int n, int E,
                    int e_lo, int e_hi, int max_blocks, int bm, hipStream_t s) {
  if (E > 256 || e_lo < 0 || e_hi > E || e_lo >= e_hi) return -1;
  if (bm != 64 && bm != 256) return -2;
  moe_align_kernel<<<1, 1024, 0, s>>>(sorted, blk_expert, n_blocks, ids, n, E, e_lo, e_hi,
                                      max_blocks, bm);
  return (int)hipGetLastError();
}

// mode 0: out = act [max_blocks*64, N=I], A = x [T, K=d], W = [E_local, 2I, d]
// mode 1: out = Y [T*k, N=d],            A = act [max_blocks*64, K=I], W = [E_local, d, I]
int omnia_moe_gemm(int mode, void* out, const void* A, const void* W, const int* sorted,
                   const int* blk_expert, const int* n_blocks, const float* route_w, int K,
                   int N, int topk, int n_assign, int e_lo, int max_blocks, hipStream_t s) {
  if (K % 64) return -1;
  if (mode == 0 ? (N % 32) : (N % 64)) return -2;
  if (max_blocks == 0) return 0;
  dim3 grid(mode == 0 ? N / 32 : N / 64, max_blocks);
  if (mode == 0)
    moe_gemm_kernel<0><<<grid, 256, 0, s>>>((bf16_t*)out, (const bf16_t*)A, (const bf16_t*)W,
                                            sorted, blk_expert, n_blocks, route_w, K, N, topk,
                                            n_assign, e_lo);
  else
    moe_gemm_kernel<1><<<grid, 256, 0, s>>>((bf16_t*)out, (const bf16_t*)A, (const bf16_t*)W,
                                            sorted, blk_expert, n_blocks, route_w, K, N, topk,
                                            n_assign, e_lo);
  return (int)hipGetLastError();
}

int omnia_moe_combine(void* out, const void* Y, const int* ids, int n_tok, int d, int topk,
                      int e_lo, int e_hi, hipStream_t s) {
  if (d % 8) return -1;
  if (n_tok == 0) return 0;
  moe_combine_kernel<<<n_tok, 256, 0, s>>>((bf16_t*)out, (const bf16_t*)Y, ids, d, topk, e_lo,
                                           e_hi);
  return (int)hipGetLastError();
}

}  // extern "C"
