// Decode-shaped projection GEMM for gfx950: out[M, N] = x[M, K] . W[N, K]^T
// with M <= 256 (one continuous-batching decode step), bf16 in, fp32 MFMA
// accumulate, bf16 out.  Replaces the hipBLASLt call on the decode hot path
// (QKV / O / gate_up / down of every layer).
//
// Why a hand kernel here: at M = 256 a GEMM is neither HBM- nor MFMA-bound by
// itself -- the per-CU load path is the limit (every column tile re-reads the
// whole x slab from L2).  The design answers that directly:
//   * BM = 64*WM rows per tile (WM in {1,2,4}); with WM covering the batch
//     every weight byte is streamed from HBM exactly once, with smaller WM the
//     row tiles of one column tile run adjacently so the re-read hits L2;
//   * wide column tiles (BN = 64*WN) keep the FLOP per staged byte high
//     (BM*BN/(BM+BN) = 85 at 256x128);
//   * split-K over S slices fills the 256 CUs when N/BN is small (QKV, O,
//     down), and the partial tiles are combined IN-LAUNCH by the last-arriving
//     slice (agent-scope release/acquire hand-off, fixed summation order, so
//     the result is deterministic and independent of XCD placement);
//   * the SwiGLU of the MLP is fused into the gate_up epilogue (MODE 1): each
//     wave's 64 columns are 32 gate rows + the matching 32 up rows of W, so
//     silu(g)*u is formed in registers and the [M, 2I] intermediate never
//     exists;
//   * 16x16x32 bf16 MFMA, LDS double buffer with the XOR-swizzled [row][8x16B]
//     image (conflict-free ds_read_b128 fragment reads), XCD-aware block
//     order so the slices of one tile share an L2.
#include "common.h"

using namespace omnia;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float4v mfma16(short8 a, short8 b, float4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// LDS image of a [rows][64] bf16 tile: chunk c (16 B) of row r at c ^ (r & 7)
__device__ __forceinline__ int swz(int row, int ch) { return row * 64 + ((ch ^ (row & 7)) << 3); }

__device__ __forceinline__ float silu(float g) { return g * __builtin_amdgcn_rcpf(1.f + __expf(-g)); }

// MODE 0: out[M, N]   = x W^T              (W: [N, K])
// MODE 1: out[M, N]   = silu(x Wg^T) * (x Wu^T), W = [Wg; Wu]: [2N, K]
template <int WM, int WN, int MODE>
__global__ __launch_bounds__(64 * WM * WN, 2) void dgemm_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
    float* __restrict__ ws, int* __restrict__ cnt, int M, int N, int K, int S, int ldo) {
  constexpr int BM = 64 * WM, BN = 64 * WN, NT = 64 * WM * WN;
  constexpr int A_CH = BM * 8 / NT, B_CH = BN * 8 / NT;  // 16-B chunks / thread / k-step
  constexpr int BUF = (BM + BN) * 64;                     // bf16 elements per stage
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * BUF];

  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  // block order: (column tile, row tile, k slice) -- a tile's slices and the row
  // tiles that share its weight columns are adjacent, i.e. on one XCD's L2
  const int mtiles = (M + BM - 1) / BM;
  const int ntile = bid / (S * mtiles);
  const int rem = bid - ntile * S * mtiles;
  const int mt = rem / S, split = rem - mt * S;
  const int tile = ntile * mtiles + mt;  // counter / slab index
  const int m0 = mt * BM;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w / WN, wn = w - wm * WN;
  const int Kb = K / S;
  const int64_t kbeg = (int64_t)split * Kb;

  const bf16_t* a_src[A_CH];
  int a_off[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    const int c = tid + i * NT, row = c >> 3, ch = c & 7;
    const int r = m0 + row < M ? m0 + row : M - 1;  // rows past the batch: clamped
    a_src[i] = X + (int64_t)r * K + kbeg + ch * 8;
    a_off[i] = swz(row, ch);
  }
  const bf16_t* b_src[B_CH];
  int b_off[B_CH];
#pragma unroll
  for (int i = 0; i < B_CH; ++i) {
    const int c = tid + i * NT, row = c >> 3, ch = c & 7;
    int64_t wrow;
    if (MODE == 0) {
      wrow = (int64_t)ntile * BN + row;
    } else {
      const int wc = row >> 6, rr = row & 63;
      const int64_t col0 = (int64_t)ntile * (32 * WN) + wc * 32;
      wrow = rr < 32 ? col0 + rr : (int64_t)N + col0 + (rr - 32);
    }
    b_src[i] = W + wrow * K + kbeg + ch * 8;
    b_off[i] = swz(row, ch);
  }

  // Two k-steps of loads in flight (register ring, depth 2) while the third is
  // computed out of LDS: at ~24 GB/s of HBM stream per CU the weight stream
  // needs >= ~64 KB outstanding per CU to cover the miss latency.
  short8 ra0[A_CH], rb0[B_CH], ra1[A_CH], rb1[B_CH];
  auto gload = [&](short8* ra, short8* rb, int k0) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) ra[i] = *reinterpret_cast<const short8*>(a_src[i] + k0);
#pragma unroll
    for (int i = 0; i < B_CH; ++i)
      rb[i] = __builtin_nontemporal_load(reinterpret_cast<const short8*>(b_src[i] + k0));
  };
  auto lstore = [&](const short8* ra, const short8* rb, int buf) {
    bf16_t* As = lds + buf * BUF;
    bf16_t* Bs = As + BM * 64;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) *reinterpret_cast<short8*>(As + a_off[i]) = ra[i];
#pragma unroll
    for (int i = 0; i < B_CH; ++i) *reinterpret_cast<short8*>(Bs + b_off[i]) = rb[i];
  };

  float4v acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = {0.f, 0.f, 0.f, 0.f};

  const int nk = Kb / 64;
  const int fr = lane & 15, fq = lane >> 4;
  auto compute = [&](int buf) {
    const bf16_t* As = lds + buf * BUF;
    const bf16_t* Bs = As + BM * 64;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      short8 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a[i] = *reinterpret_cast<const short8*>(As + swz(wm * 64 + 16 * i + fr, ks * 4 + fq));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        b[j] = *reinterpret_cast<const short8*>(Bs + swz(wn * 64 + 16 * j + fr, ks * 4 + fq));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(a[i], b[j], acc[i][j]);
    }
  };
  // Branch-free load/store schedule: every iteration issues its prefetch (the
  // k offset is clamped at the tail, re-reading the last slice harmlessly) and
  // writes its staging buffer, so hipcc can count vmcnt across the loop instead
  // of draining every outstanding load before the next prefetch (which had
  // serialised the k-steps on the full memory latency).
  const int klast = (nk - 1) * 64;
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

  if (S > 1) {
    // ---- in-launch split-K combine (release -> ticket -> acquire) ----
    float4v* slab = reinterpret_cast<float4v*>(ws) + (int64_t)tile * S * 16 * NT;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) slab[((int64_t)split * 16 + i * 4 + j) * NT + tid] = acc[i][j];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(lds);  // the one LDS array (no second __shared__)
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int old = __hip_atomic_fetch_add(&cnt[tile], 1, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == S - 1;
      if (last) {
        cnt[tile] = 0;  // ready for the next launch (stream-ordered)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    // fixed order s = 0..S-1 -> bitwise identical whatever slice arrives last
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float4v sm[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) sm[j] = {0.f, 0.f, 0.f, 0.f};
      for (int s = 0; s < S; ++s) {
        float4v v[4];
        if (s == split) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = acc[i][j];
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = slab[((int64_t)s * 16 + i * 4 + j) * NT + tid];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) sm[j] += v[j];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = sm[j];
    }
  }

  // ---- epilogue: lane holds rows wm*64 + 16i + 4fq + r, columns 16j + fr of its wave tile
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + wm * 64 + 16 * i + 4 * fq + r;
      if (row >= M) continue;
      bf16_t* orow = out + (int64_t)row * ldo;
      if (MODE == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          orow[(int64_t)ntile * BN + wn * 64 + 16 * j + fr] = f2bf(acc[i][j][r]);
      } else {
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
          orow[(int64_t)ntile * (32 * WN) + wn * 32 + 16 * jj + fr] =
              f2bf(silu(acc[i][jj][r]) * acc[i][jj + 2][r]);
      }
    }
  }
}

template <int WM, int WN, int MODE>
int launch(bf16_t* out, const bf16_t* X, const bf16_t* W, float* ws, int* cnt, int M, int N,
           int K, int S, int ldo, hipStream_t s) {
  const int cols = MODE == 0 ? 64 * WN : 32 * WN;
  const int tiles = (N / cols) * ((M + 64 * WM - 1) / (64 * WM));
  dgemm_kernel<WM, WN, MODE><<<tiles * S, 64 * WM * WN, 0, s>>>(out, X, W, ws, cnt, M, N, K, S,
                                                                 ldo);
  return (int)hipGetLastError();
}

template <int MODE>
int dispatch(int wm, int wn, bf16_t* out, const bf16_t* X, const bf16_t* W, float* ws, int* cnt,
             int M, int N, int K, int S, int ldo, hipStream_t s) {
#define OMNIA_DG(a, b) \
  if (wm == a && wn == b) return launch<a, b, MODE>(out, X, W, ws, cnt, M, N, K, S, ldo, s);
  OMNIA_DG(1, 1) OMNIA_DG(1, 2) OMNIA_DG(1, 4)
  OMNIA_DG(2, 1) OMNIA_DG(2, 2) OMNIA_DG(2, 4)
  OMNIA_DG(4, 1) OMNIA_DG(4, 2)
#undef OMNIA_DG
  return -10;
}

}  // namespace

extern "C" {

// Returns 0 on success, <0 on a shape the kernel does not cover (checked BEFORE
// any launch).  ws must hold tiles*S*BM*BN floats when S > 1; cnt >= tiles ints,
// zero on first use (the combining block re-zeroes its counter).
int omnia_dgemm(int mode, void* out, const void* X, const void* W, float* ws, int* cnt, int M,
                int N, int K, int S, int wm, int wn, int ldo, int64_t ws_floats, int cnt_len,
                hipStream_t s) {
  if (mode != 0 && mode != 1) return -1;
  if (M < 1 || M > 256) return -2;
  if (S < 1 || K % (64 * S)) return -3;
  const int cols = mode == 0 ? 64 * wn : 32 * wn;
  if (N % cols) return -4;
  const int tiles = (N / cols) * ((M + 64 * wm - 1) / (64 * wm));
  if (S > 1) {
    if (tiles > cnt_len) return -5;
    if ((int64_t)tiles * S * (64 * wm) * (64 * wn) > ws_floats) return -6;
  }
  if ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W)) & 15) return -7;
  if (ldo < (mode == 0 ? N : N)) return -8;
  if (mode == 0)
    return dispatch<0>(wm, wn, (bf16_t*)out, (const bf16_t*)X, (const bf16_t*)W, ws, cnt, M, N,
                       K, S, ldo, s);
  return dispatch<1>(wm, wn, (bf16_t*)out, (const bf16_t*)X, (const bf16_t*)W, ws, cnt, M, N, K,
                     S, ldo, s);
}

}  // extern "C"
