// Wide-batch weight-streaming decode GEMM for gfx950: out[M, N] = x[M, K] . W[N, K]^T
// for 128 < M <= 256 (the full continuous batch of a decode step), bf16 in, fp32
// accumulate on v_mfma_f32_32x32x16_bf16.  SURVEY §2.4 K3 / K8 / K9 / K10.
//
// At M = 256 a Llama-3-8B projection sits on the ridge: 256 FLOP per weight byte
// against ~310 FLOP/B for MI355X (2.5 PF / 8 TB/s), so streaming W at HBM speed
// needs ~55 % of MFMA peak WHILE every CU also pulls its share of x.  wgemm.hip's
// 16x16x32 design loses there because each block covers only 32-64 weight rows:
// it re-stages the whole 2 MB x slab per block (4x the weight bytes through
// L2 -> LDS) and feeds one 1 KB A fragment to just NW = 2 MFMAs.  This kernel
// turns both ratios around:
//   * one wave per SIMD (4 per block, __launch_bounds__(256, 1)) owns ALL M rows x
//     32*WT weight rows: an 8 x WT grid of 32x32 accumulators (256 AGPRs at WT=2),
//     so a block covers 128*WT weight rows and x crosses L2 -> LDS once per
//     128*WT rows instead of once per 32-64;
//   * each ds_read_b128 A fragment feeds WT 32x32x16 MFMAs (32 cycles each):
//     at WT = 2 that is one LDS read per 64 MFMA cycles, far from the LDS limit;
//   * W goes HBM -> B-fragment registers with no LDS hop: lane (n = l&31,
//     h = l>>5) reads 64 contiguous bytes of weight row n per 64-k stage (k =
//     32h .. 32h+31) as four 16-B loads, and the K index inside each MFMA is
//     permuted to match (substep j uses k = 32h + 8j + e), so a stage's four
//     load instructions cover 32 rows x 128 B = whole cache lines.  A 4-stage
//     register ring (nontemporal, so W does not evict the L2-resident x) keeps
//     ~24 KB of weights in flight per wave;
//   * x stages are 256 rows x 64 k (32 KB) in an XOR-swizzled LDS image, double
//     buffered, loaded one stage ahead into registers.
// Epilogues (MODE) as in wgemm.hip: 0 bf16, 1 SwiGLU (tile 0 = gate, tile 1 = up
// columns of the same output features), 2 fp32 split-K slabs reduced by the
// consumer kernel (splitk.hip).
#include "common.h"

using namespace omnia;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float16v mfma32(short8 a, short8 b, float16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// [rows][64] bf16 stage image: 16-B chunk c of row r stored at c ^ (r & 7)
__device__ __forceinline__ int swz(int row, int ch) { return row * 64 + ((ch ^ (row & 7)) << 3); }

__device__ __forceinline__ float silu(float g) { return g * __builtin_amdgcn_rcpf(1.f + __expf(-g)); }

constexpr int kRing = 4;  // W register ring depth (stages of 64 k)

template <int MT, int WT, int MODE>
__global__ __launch_bounds__(256, 1) void wgemm_wide_kernel(
    void* __restrict__ out, const bf16_t* __restrict__ X, const bf16_t* __restrict__ W, int M,
    int N, int K, int S, int ldo) {
  constexpr int MP = 32 * MT;      // padded batch rows
  constexpr int WROWS = 32 * WT;   // weight rows per wave
  constexpr int XCH = MP * 8;      // 16-B chunks of one x stage
  constexpr int XPT = XCH / 256;   // chunks per thread (MP is a multiple of 32)
  constexpr int BUF = MP * 64;
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * BUF];

  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = bid / S, split = bid - tile * S;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int fn = lane & 31, fh = lane >> 5;
  const int Kb = K / S;
  const int64_t kbeg = (int64_t)split * Kb;
  const int wave_id = tile * 4 + wv;

  // ---- x staging: thread owns chunks c = tid + 256 i (row c >> 3, chunk c & 7)
  const bf16_t* xs[XPT];
  int xo[XPT];
#pragma unroll
  for (int i = 0; i < XPT; ++i) {
    const int c = tid + i * 256;
    const int row = c >> 3, ch = c & 7;
    const int r = row < M ? row : M - 1;  // padded rows are copies, never stored
    xs[i] = X + (int64_t)r * K + kbeg + ch * 8;
    xo[i] = swz(row, ch);
  }
  // ---- this wave's weight rows: lane reads 64 B of row (.. + fn) at k = 32 fh
  const bf16_t* wsrc[WT];
#pragma unroll
  for (int t = 0; t < WT; ++t) {
    int64_t row;
    if (MODE == 1) {  // tile 0: gate features, tile 1: the same up features
      const int64_t oc0 = (int64_t)wave_id * 32;
      row = t == 0 ? oc0 + fn : (int64_t)N + oc0 + fn;
    } else {
      row = (int64_t)wave_id * WROWS + 32 * t + fn;
    }
    wsrc[t] = W + row * K + kbeg + fh * 32;
  }

  short8 wr[kRing][WT][4];
  short8 xr[XPT];
  float16v acc[MT][WT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int t = 0; t < WT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][t][r] = 0.f;

  auto wload = [&](short8 (&w)[WT][4], int k) {
#pragma unroll
    for (int t = 0; t < WT; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        w[t][j] = __builtin_nontemporal_load(
            reinterpret_cast<const short8*>(wsrc[t] + k + 8 * j));
  };
  auto xload = [&](int k) {
#pragma unroll
    for (int i = 0; i < XPT; ++i) xr[i] = *reinterpret_cast<const short8*>(xs[i] + k);
  };
  auto xstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < XPT; ++i)
      *reinterpret_cast<short8*>(lds + buf * BUF + xo[i]) = xr[i];
  };
  auto compute = [&](int buf, short8 (&w)[WT][4]) {
    const bf16_t* As = lds + buf * BUF;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        // A[row 32i + fn][k = 32 fh + 8 j .. +8]: chunk 4 fh + j of the stage row
        const short8 a = *reinterpret_cast<const short8*>(As + swz(32 * i + fn, 4 * fh + j));
#pragma unroll
        for (int t = 0; t < WT; ++t) acc[i][t] = mfma32(a, w[t][j], acc[i][t]);
      }
  };

  // Branch-free schedule over nk (multiple of kRing, host-checked) 64-k stages:
  // stage s consumes ring slot s % kRing and refills it with stage s + kRing
  // (clamped at the tail: re-reads the last stage harmlessly), while the next
  // x stage is published into the other LDS buffer behind one barrier.
  const int nk = Kb / 64, klast = (nk - 1) * 64;
#pragma unroll
  for (int s = 0; s < kRing; ++s) wload(wr[s], min(64 * s, klast));
  xload(0);
  xstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; kt += kRing) {
#pragma unroll
    for (int u = 0; u < kRing; ++u) {
      xload(min((kt + u + 1) * 64, klast));
      compute(u & 1, wr[u]);
      wload(wr[u], min((kt + u + kRing) * 64, klast));
      xstore((u + 1) & 1);
      __syncthreads();
    }
  }

  // ---- epilogue: acc[i][t][r] = out[row 32i + (r&3) + 8(r>>2) + 4 fh][col 32t + fn]
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = 32 * i + (r & 3) + 8 * (r >> 2) + 4 * fh;
      if (row >= M) continue;
      if (MODE == 0) {
        bf16_t* o = reinterpret_cast<bf16_t*>(out) + (int64_t)row * ldo +
                    (int64_t)wave_id * WROWS + fn;
#pragma unroll
        for (int t = 0; t < WT; ++t) o[32 * t] = f2bf(acc[i][t][r]);
      } else if (MODE == 1) {
        bf16_t* o = reinterpret_cast<bf16_t*>(out) + (int64_t)row * ldo +
                    (int64_t)wave_id * 32 + fn;
        o[0] = f2bf(silu(acc[i][0][r]) * acc[i][1][r]);
      } else {
        float* o = reinterpret_cast<float*>(out) + ((int64_t)split * M + row) * ldo +
                   (int64_t)wave_id * WROWS + fn;
#pragma unroll
        for (int t = 0; t < WT; ++t) o[32 * t] = acc[i][t][r];
      }
    }
}

template <int MT, int MODE>
int launch_wt(void* out, const bf16_t* X, const bf16_t* W, int M, int N, int K, int S, int ldo,
              int wt, hipStream_t s) {
  const int wrows = MODE == 1 ? 2 * N : N;
  const int tiles = wrows / (128 * wt);
  if (wt == 2) {
    wgemm_wide_kernel<MT, 2, MODE><<<tiles * S, 256, 0, s>>>(out, X, W, M, N, K, S, ldo);
  } else if constexpr (MODE != 1) {
    if (wt != 1) return -20;
    wgemm_wide_kernel<MT, 1, MODE><<<tiles * S, 256, 0, s>>>(out, X, W, M, N, K, S, ldo);
  } else {
    return -20;
  }
  return (int)hipGetLastError();
}

template <int MODE>
int launch_mode(void* out, const bf16_t* X, const bf16_t* W, int M, int N, int K, int S, int ldo,
                int wt, hipStream_t s) {
  if (M <= 192) return launch_wt<6, MODE>(out, X, W, M, N, K, S, ldo, wt, s);
  return launch_wt<8, MODE>(out, X, W, M, N, K, S, ldo, wt, s);
}

}  // namespace

extern "C" {

// Returns 0 on success, < 0 for a shape the kernel does not cover (checked
// BEFORE any launch).  mode 2 writes S fp32 slabs of [M, ldo].
int omnia_wgemm_wide(int mode, void* out, const void* X, const void* W, int M, int N, int K,
                     int S, int wt, int ldo, hipStream_t s) {
  if (mode < 0 || mode > 2) return -1;
  if (M < 129 || M > 256) return -2;
  if (S < 1 || K % (64 * kRing * S)) return -3;  // whole ring turns of 64-k stages per slice
  if (wt != 1 && wt != 2) return -4;
  if (mode == 1 && wt != 2) return -5;
  const int wrows = mode == 1 ? 2 * N : N;
  if (wrows % (128 * wt)) return -7;
  if (mode == 1 && N % 128) return -8;
  if (mode != 2 && S != 1) return -9;
  if ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W)) & 15) return -10;
  if (ldo < N) return -11;
  const bf16_t* x = (const bf16_t*)X;
  const bf16_t* w = (const bf16_t*)W;
  if (mode == 0) return launch_mode<0>(out, x, w, M, N, K, S, ldo, wt, s);
  if (mode == 1) return launch_mode<1>(out, x, w, M, N, K, S, ldo, wt, s);
  return launch_mode<2>(out, x, w, M, N, K, S, ldo, wt, s);
}

}  // extern "C"
