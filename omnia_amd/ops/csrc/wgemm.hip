// Weight-streaming decode GEMM for gfx950: out[M, N] = x[M, K] . W[N, K]^T with
// M <= 256 (one decode step of the continuous batch), bf16 in, fp32 MFMA
// accumulate.  SURVEY §2.4 K3 / K8 / K9 / K10 / K11.
//
// Decode projections at M = 256 are balanced between three limits (per layer
// of Llama-3-8B: 111 GFLOP of MFMA work, 436 MB of weights, and the L2 -> CU
// operand traffic).  The earlier design (gemm.hip) staged BOTH operands through
// LDS with 64 x 64 wave tiles: every weight byte crossed the LDS write + read
// path and every column tile re-read the whole x slab, so the per-CU load path
// -- not HBM -- set the speed (1.4-3.1 TB/s).  Here the roles are split by
// reuse:
//   * W (used once) goes straight from HBM into MFMA B-fragment registers:
//     lane l loads 16 B of W row (n0 + 16j + (l & 15)) at k-group (l >> 4), which
//     is exactly the 16x16x32 B-operand layout, nontemporal so it does not
//     evict the L2-resident x.  A 2-stage register ring keeps the next 64-k
//     stage of every wave's rows in flight while the current one is consumed.
//   * x (re-used by every wave) is staged once per 64-k stage into an
//     XOR-swizzled LDS image shared by the block's waves and read with
//     conflict-free ds_read_b128 A-fragments.
//   * each wave owns 16*NW weight rows x ALL M rows, so a weight byte is
//     fetched from HBM exactly once and the LDS bytes per MFMA shrink as NW
//     grows (1 KB / NW per 16x16x32 MFMA).
// Epilogues (MODE):
//   0  bf16 out[M, ldo]
//   1  SwiGLU: the wave's rows are NW/2 gate fragments + the matching NW/2 up
//      fragments, silu(g) * u formed in registers (no [M, 2I] intermediate)
//   2  fp32 split-K partial slab part[split][M][ldo]; the NEXT kernel reduces
//      the S slices while doing its own work (RoPE + KV write for QKV, residual
//      add + RMSNorm for O / down: splitk_epilogue.hip), so split-K costs no
//      extra launch, no atomics and no inter-block hand-off.
#include "common.h"

using namespace omnia;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float4v mfma16(short8 a, short8 b, float4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// [rows][64] bf16 stage image: 16-B chunk c of row r stored at c ^ (r & 7)
__device__ __forceinline__ int swz(int row, int ch) { return row * 64 + ((ch ^ (row & 7)) << 3); }

__device__ __forceinline__ float silu(float g) { return g * __builtin_amdgcn_rcpf(1.f + __expf(-g)); }

template <int MF, int NW, int MODE, int NWAVES>
__global__ __launch_bounds__(64 * NWAVES, 1) void wgemm_kernel(
    void* __restrict__ out, const bf16_t* __restrict__ X, const bf16_t* __restrict__ W, int M,
    int N, int K, int S, int ldo) {
  constexpr int MP = 16 * MF;            // padded batch rows
  constexpr int NT = 64 * NWAVES;
  constexpr int WROWS = 16 * NW;         // weight rows per wave
  constexpr int XCH = MP * 8;            // 16-B chunks of one x stage (MP x 64 bf16)
  constexpr int XPT = (XCH + NT - 1) / NT;
  constexpr int BUF = MP * 64;
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * BUF];

  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = bid / S, split = bid - tile * S;  // a tile's slices are adjacent
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int Kb = K / S;
  const int64_t kbeg = (int64_t)split * Kb;
  const int wave_id = tile * NWAVES + wv;

  // ---- x staging addresses (rows past the batch are clamped; never stored)
  const bf16_t* xs[XPT];
  int xo[XPT];
#pragma unroll
  for (int i = 0; i < XPT; ++i) {
    const int c = tid + i * NT;
    const int row = (c < XCH ? c : 0) >> 3, ch = c & 7;
    const int r = row < M ? row : M - 1;
    xs[i] = X + (int64_t)r * K + kbeg + ch * 8;
    xo[i] = swz(row, ch);
  }
  // ---- this wave's weight rows
  const bf16_t* wsrc[NW];
#pragma unroll
  for (int j = 0; j < NW; ++j) {
    int64_t row;
    if (MODE == 1) {
      const int64_t oc0 = (int64_t)wave_id * (WROWS / 2);
      row = j < NW / 2 ? oc0 + 16 * j + fr : (int64_t)N + oc0 + 16 * (j - NW / 2) + fr;
    } else {
      row = (int64_t)wave_id * WROWS + 16 * j + fr;
    }
    wsrc[j] = W + row * K + kbeg + fq * 8;
  }

  short8 wa[NW][2], wb[NW][2], xr[XPT];
  float4v acc[MF][NW];
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int j = 0; j < NW; ++j) acc[i][j] = {0.f, 0.f, 0.f, 0.f};

  auto wload = [&](short8 (&w)[NW][2], int k) {
#pragma unroll
    for (int j = 0; j < NW; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        w[j][h] = __builtin_nontemporal_load(
            reinterpret_cast<const short8*>(wsrc[j] + k + 32 * h));
  };
  auto xload = [&](int k) {
#pragma unroll
    for (int i = 0; i < XPT; ++i)
      if (XPT * NT == XCH || tid + i * NT < XCH)
        xr[i] = *reinterpret_cast<const short8*>(xs[i] + k);
  };
  auto xstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < XPT; ++i)
      if (XPT * NT == XCH || tid + i * NT < XCH)
        *reinterpret_cast<short8*>(lds + buf * BUF + xo[i]) = xr[i];
  };
  auto compute = [&](int buf, short8 (&w)[NW][2]) {
    const bf16_t* As = lds + buf * BUF;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        const short8 a = *reinterpret_cast<const short8*>(As + swz(16 * i + fr, h * 4 + fq));
#pragma unroll
        for (int j = 0; j < NW; ++j) acc[i][j] = mfma16(a, w[j][h], acc[i][j]);
      }
  };

  // Branch-free schedule over an even number of 64-k stages (host-checked):
  // every half-iteration issues the next x stage, consumes one W ring slot,
  // refills that slot two stages ahead (clamped at the tail: re-reads the last
  // stage harmlessly) and publishes the next x stage behind one barrier.
  const int nk = Kb / 64, klast = (nk - 1) * 64;
  wload(wa, 0);
  wload(wb, min(64, klast));
  xload(0);
  xstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; kt += 2) {
    xload(min((kt + 1) * 64, klast));
    compute(0, wa);
    wload(wa, min((kt + 2) * 64, klast));
    xstore(1);
    __syncthreads();
    xload(min((kt + 2) * 64, klast));
    compute(1, wb);
    wload(wb, min((kt + 3) * 64, klast));
    xstore(0);
    __syncthreads();
  }

  // ---- epilogue: lane holds rows 16i + 4fq + r, columns 16j + fr of its wave
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * i + 4 * fq + r;
      if (row >= M) continue;
      if (MODE == 0) {
        bf16_t* o = reinterpret_cast<bf16_t*>(out) + (int64_t)row * ldo + (int64_t)wave_id * WROWS;
#pragma unroll
        for (int j = 0; j < NW; ++j) o[16 * j + fr] = f2bf(acc[i][j][r]);
      } else if (MODE == 1) {
        bf16_t* o = reinterpret_cast<bf16_t*>(out) + (int64_t)row * ldo +
                    (int64_t)wave_id * (WROWS / 2);
#pragma unroll
        for (int j = 0; j < NW / 2; ++j)
          o[16 * j + fr] = f2bf(silu(acc[i][j][r]) * acc[i][j + NW / 2][r]);
      } else {
        float* o = reinterpret_cast<float*>(out) + ((int64_t)split * M + row) * ldo +
                   (int64_t)wave_id * WROWS;
#pragma unroll
        for (int j = 0; j < NW; ++j) o[16 * j + fr] = acc[i][j][r];
      }
    }
}

template <int MF, int NW, int MODE>
int launch_nw(void* out, const bf16_t* X, const bf16_t* W, int M, int N, int K, int S, int ldo,
              int nwaves, hipStream_t s) {
  const int rows_per_block = 16 * NW * nwaves;
  const int wrows = MODE == 1 ? 2 * N : N;
  const int tiles = wrows / rows_per_block;
  if (nwaves == 4) {
    wgemm_kernel<MF, NW, MODE, 4><<<tiles * S, 256, 0, s>>>(out, X, W, M, N, K, S, ldo);
  } else if (nwaves == 2) {
    wgemm_kernel<MF, NW, MODE, 2><<<tiles * S, 128, 0, s>>>(out, X, W, M, N, K, S, ldo);
  } else {
    return -20;
  }
  return (int)hipGetLastError();
}

template <int MF, int MODE>
int launch_mf(void* out, const bf16_t* X, const bf16_t* W, int M, int N, int K, int S, int ldo,
              int nw, int nwaves, hipStream_t s) {
  if constexpr (MODE != 1) {
    if (nw == 1) return launch_nw<MF, 1, MODE>(out, X, W, M, N, K, S, ldo, nwaves, s);
  }
  if (nw == 2) return launch_nw<MF, 2, MODE>(out, X, W, M, N, K, S, ldo, nwaves, s);
  if constexpr (MF <= 8) {  // 4 fragments per wave x > 128 rows spills the accumulators
    if (nw == 4) return launch_nw<MF, 4, MODE>(out, X, W, M, N, K, S, ldo, nwaves, s);
  }
  return -21;
}

template <int MODE>
int launch_mode(void* out, const bf16_t* X, const bf16_t* W, int M, int N, int K, int S, int ldo,
                int nw, int nwaves, hipStream_t s) {
  const int mf = (M + 15) / 16;
#define OMNIA_WG(F) \
  if (mf <= F) return launch_mf<F, MODE>(out, X, W, M, N, K, S, ldo, nw, nwaves, s);
  OMNIA_WG(1) OMNIA_WG(2) OMNIA_WG(4) OMNIA_WG(6) OMNIA_WG(8) OMNIA_WG(12) OMNIA_WG(16)
#undef OMNIA_WG
  return -22;
}

}  // namespace

extern "C" {

// Returns 0 on success, < 0 for a shape the kernel does not cover (checked
// BEFORE any launch).  mode 2 writes S fp32 slabs of [M, ldo].
int omnia_wgemm(int mode, void* out, const void* X, const void* W, int M, int N, int K, int S,
                int nw, int nwaves, int ldo, hipStream_t s) {
  if (mode < 0 || mode > 2) return -1;
  if (M < 1 || M > 256) return -2;
  if (S < 1 || K % (128 * S)) return -3;  // an even number of 64-k stages per slice
  if (mode == 1 && (nw % 2)) return -4;
  if (nw != 1 && nw != 2 && nw != 4) return -5;
  if (nwaves != 2 && nwaves != 4) return -6;
  const int wrows = mode == 1 ? 2 * N : N;
  const int per_block = 16 * nw * nwaves;
  if (wrows % per_block) return -7;
  if (mode == 1 && N % (8 * nw * nwaves)) return -8;
  if (mode != 2 && S != 1) return -9;
  if ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W)) & 15) return -10;
  if (ldo < N) return -11;
  const bf16_t* x = (const bf16_t*)X;
  const bf16_t* w = (const bf16_t*)W;
  if (mode == 0) return launch_mode<0>(out, x, w, M, N, K, S, ldo, nw, nwaves, s);
  if (mode == 1) return launch_mode<1>(out, x, w, M, N, K, S, ldo, nw, nwaves, s);
  return launch_mode<2>(out, x, w, M, N, K, S, ldo, nw, nwaves, s);
}

}  // extern "C"
