// Full-batch tile GEMM for decode projections on gfx950:
//   out = x[M, K] . W[N, K]^T   for 129 <= M <= 256 (one continuous-batching
// decode step) and, tiled 256 rows at a time, any larger M (prefill chunks:
// MODE 1 then fuses SwiGLU into the prefill gate_up GEMM); bf16 operands, fp32
// MFMA accumulate.  SURVEY §2.4 K3/K8/K9/K10.
//
// At M = 256 a Llama-3-8B projection sits on the MI355X ridge (256 FLOP per
// weight byte vs ~400 FLOP/B of dense bf16 peak over achievable HBM), so the
// kernel has to keep the matrix cores busy WHILE the weights stream at HBM
// speed.  The per-CU limit is the load path, not HBM: every column tile
// re-reads its x slab from L2.  The design therefore maximises FLOP per staged
// byte and keeps the staging pipeline full:
//   * one block owns ALL 256 batch rows x BN weight rows (BN = 64/128/256), so
//     W crosses HBM -> LDS exactly once and x crosses L2 -> LDS once per BN
//     weight rows (BM*BN/(BM+BN) = 85 FLOP/B at BN = 128, 128 at BN = 256);
//   * both operands go global -> LDS by direct LDS-DMA (global_load_lds_dwordx4,
//     16 B per lane, 1 KB = 8 rows x 128 B per wave instruction).  The LDS image
//     is lane-linear; the bank-conflict XOR swizzle (chunk c of row r at
//     c ^ (r & 7)) is applied to the per-lane SOURCE address and to the
//     fragment reads (the same involution);
//   * NS-deep LDS ring (NS = 4/3/2 stages of 64 k for BN = 64/128/256, as many
//     as 160 KB allows) with a COUNTED `s_waitcnt vmcnt` and raw `s_barrier`,
//     so NS-2 stages of loads stay in flight across every barrier -- hipcc's
//     __syncthreads() would drain them (vmcnt(0)) on every k-step;
//   * 8 waves (512 threads) on 16x16x32 bf16 MFMA, wave tile 64x64 (BN 128),
//     128x64 (BN 256) or 64x32 (BN 64);
//   * split-K over S slices (uneven splits allowed) fills the 256 CUs; slices
//     write fp32 partial slabs [S][M][N] that the NEXT kernel reduces as part of
//     its own work (splitk.hip: QKV -> RoPE + paged KV write, O / down ->
//     residual add + RMSNorm, gate_up -> SwiGLU), so no combine launch exists;
//   * MODE 1 fuses SwiGLU into the epilogue (S = 1): each wave's BN/2 columns
//     are gate features and the matching up features of W = [Wg; Wu];
//   * block order: XCD-remapped, split-major, so the blocks sharing an XCD's L2
//     mostly share one x slice.
// MODE 0: bf16 out[M, ldo]; MODE 1: bf16 SwiGLU out[M, ldo] (N = features);
// MODE 2: fp32 partial slabs out[S][M][N]; MODE 3: the same slabs in fp16.
#include <type_traits>

#include "common.h"

using namespace omnia;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ float4v mfma16(short8 a, short8 b, float4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}


__device__ __forceinline__ float silu(float g) { return g * __builtin_amdgcn_rcpf(1.f + __expf(-g)); }

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// BK = 64: stages of 64 k (8 x 16-B chunks per row, chunk c of row r at
// c ^ (r & 7)); BK = 32: half-size stages (4 chunks per row at c ^ ((r >> 2) & 3),
// conflict-free for the 16 rows x 16 B a ds_read_b128 quarter-wave reads), so the
// ring holds twice as many stages and ~2x the bytes stay in flight per CU -- the
// per-CU L2 -> LDS intake is latency x bytes in flight.
template <int BK>
__device__ __forceinline__ int swz(int row, int ch) {
  return BK == 64 ? row * 64 + ((ch ^ (row & 7)) << 3)
                  : row * 32 + ((ch ^ ((row >> 2) & 3)) << 3);
}

template <int BN, int BK_>
struct Geo {
  static constexpr int BM = 256, BK = BK_;
  static constexpr int WGN = BN >= 256 ? 4 : 2;  // waves along N
  static constexpr int WGM = 8 / WGN;
  static constexpr int WTM = BM / WGM, WTN = BN / WGN;
  static constexpr int FM = WTM / 16, FN = WTN / 16;
  static constexpr int STAGE = (BM + BN) * BK;                  // bf16 elements per stage
  static constexpr int NS_FIT = (160 * 1024) / (STAGE * 2);
  static constexpr int NS_MAX = BK == 64 ? 4 : 8;
  static constexpr int NS = NS_FIT > NS_MAX ? NS_MAX : NS_FIT;  // LDS ring depth
  static constexpr int CH = BK / 8;                             // 16-B chunks per row
  static constexpr int RPI = 64 / CH;                           // rows per wave instruction
  static constexpr int A_IN = BM / (8 * RPI), B_IN = BN / (8 * RPI);  // glds per wave per stage
  static constexpr int L = A_IN + B_IN;
  static_assert(A_IN * 8 * RPI == BM && B_IN * 8 * RPI == BN, "stage rows per wave");
  static_assert(NS >= 2, "ring too shallow");
};

// PIPE = 1 (BK = 64, BN <= 128): the LDS -> register fragment reads of stage t+1
// are issued right after stage t+1's barrier and run under stage t's MFMAs
// (fragments double-buffered in registers), instead of all 8 waves bursting their
// reads after each barrier and then waiting on them; the ring also keeps one more
// stage in flight, since a stage's buffer is free as soon as its fragments are
// in registers.
// PK: W is tile-packed (ops.tgemm_pack): [tile][k-step][BN rows][64], rows in
// this kernel's tile order and each row's 16-B chunks pre-permuted by the LDS
// swizzle, so a stage's weights are ONE contiguous BN x 128 B run that the
// LDS-DMA reads lane-linearly.  Row-major W hands every stage 128-B pieces of BN
// rows 2*K bytes apart: that pattern streams at ~4.5 TB/s, the packed one at
// ~6.0 TB/s (scripts/microbench/w_depth.hip, profiles/r5/decode_gemm/).
template <int BN, int MODE, int WNT, int BK, int PIPE, int PK = 0>
__global__ __launch_bounds__(512, 2) void tgemm_kernel(void* __restrict__ out,
                                                       const bf16_t* __restrict__ X,
                                                       const bf16_t* __restrict__ W, int M, int N,
                                                       int K, int S, int ldo) {
  using G = Geo<BN, BK>;
  constexpr int NS = G::NS, L = G::L, A_IN = G::A_IN, B_IN = G::B_IN;
  constexpr int CH = G::CH, RPI = G::RPI;
  constexpr int FM = G::FM, FN = G::FN, WTM = G::WTM, WTN = G::WTN;
  __shared__ __attribute__((aligned(16))) bf16_t lds[NS * G::STAGE];

  // mode 1 tiles hold BN/2 output features (gate + up rows of W)
  const int ntiles = MODE == 1 ? N / (BN / 2) : N / BN;
  const int bid0 = xcd_remap(blockIdx.x, gridDim.x);
  // M > 256 (prefill): 256-row tiles, grouped GM at a time per (split, tile) so
  // consecutive blocks -- one XCD after the remap -- share the W tile in L2
  const int per_m = ntiles * S, mtiles = (M + 255) >> 8;
  int mt = 0, bid = bid0;
  if (mtiles > 1) {
    constexpr int GM = 4;
    const int g = bid0 / (GM * per_m), gm0 = g * GM;
    const int gsz = mtiles - gm0 < GM ? mtiles - gm0 : GM;
    const int idx = bid0 - gm0 * per_m;
    mt = gm0 + idx % gsz;
    bid = idx / gsz;
  }
  const int split = bid / ntiles, tile = bid - split * ntiles;
  const int m0 = mt << 8, Mt = M - m0 < 256 ? M - m0 : 256;  // rows of this tile
  const int nk = K / BK;
  const int kb = split * nk / S, ke = (split + 1) * nk / S;
  const int n_loc = ke - kb;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / G::WGN, wn = w - wm * G::WGN;

  // ---- per-lane LDS-DMA sources: instruction i of this wave covers RPI rows; lane
  // l fills row RPI*i' + l / CH, LDS chunk l % CH <- the global chunk that the
  // swizzle places there (the XOR is an involution: swz<BK>(row, c) position)
  const int lr = lane / CH, lp = lane % CH;
  auto gchunk = [&](int row) { return BK == 64 ? lp ^ (row & 7) : lp ^ ((row >> 2) & 3); };
  const bf16_t* a_src[A_IN];
#pragma unroll
  for (int i = 0; i < A_IN; ++i) {
    const int row = RPI * (w * A_IN + i) + lr;
    const int r = row < Mt ? row : Mt - 1;  // rows past the batch: clamped copies, never stored
    a_src[i] = X + (int64_t)(m0 + r) * K + (int64_t)kb * BK + gchunk(row) * 8;
  }
  const bf16_t* b_src[B_IN];
#pragma unroll
  for (int i = 0; i < B_IN; ++i) {
    const int rr = RPI * (w * B_IN + i) + lr;  // row of the B tile
    int64_t wrow;
    if (MODE == 1) {
      const int wv = rr / WTN, q = rr - wv * WTN;
      const int64_t f0 = (int64_t)tile * (BN / 2) + wv * (WTN / 2);
      wrow = q < WTN / 2 ? f0 + q : (int64_t)N + f0 + (q - WTN / 2);
    } else {
      wrow = (int64_t)tile * BN + rr;
    }
    b_src[i] = PK ? W + ((int64_t)tile * (K / BK) + kb) * BN * BK + rr * BK + lp * 8
                  : W + wrow * K + (int64_t)kb * BK + gchunk(rr) * 8;
  }
  constexpr int64_t WSTEP = PK ? BN * BK : BK;  // W elements per k-stage
  const int a_dst0 = (RPI * w * A_IN) * BK;              // element offsets inside a stage
  const int b_dst0 = 256 * BK + (RPI * w * B_IN) * BK;

  auto issue = [&](int stage, int kl) {
    bf16_t* base = lds + stage * G::STAGE;
    const int koff = kl * BK;
#pragma unroll
    for (int i = 0; i < A_IN; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(a_src[i] + koff),
                                       (lds_ptr_t)(base + a_dst0 + i * 512), 16, 0, 0);
#pragma unroll
    for (int i = 0; i < B_IN; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(b_src[i] + kl * WSTEP),
                                       (lds_ptr_t)(base + b_dst0 + i * 512), 16, 0,
                                       WNT ? 2 : 0);
  };

  float4v acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = {0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  // both 32-k halves of the stage are read up front, so the second half's LDS
  // reads are in flight under the first half's MFMAs (counted lgkmcnt by hipcc)
  constexpr int KS = BK / 32;  // 32-k MFMA steps per stage
  auto compute = [&](int stage) {
    const bf16_t* As = lds + stage * G::STAGE;
    const bf16_t* Bs = As + 256 * BK;
    short8 a[KS][FM], b[KS][FN];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int j = 0; j < FN; ++j)
        b[ks][j] = *reinterpret_cast<const short8*>(Bs + swz<BK>(wn * WTN + 16 * j + fr,
                                                                 ks * 4 + fq));
#pragma unroll
      for (int i = 0; i < FM; ++i)
        a[ks][i] = *reinterpret_cast<const short8*>(As + swz<BK>(wm * WTM + 16 * i + fr,
                                                                 ks * 4 + fq));
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(a[ks][i], b[ks][j], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
  };

  const int klast = n_loc - 1;
  if constexpr (PIPE) {
    static_assert(BK == 64 && BN <= 128, "register-pipelined variant: BK 64, BN <= 128");
    auto ldfrag = [&](int stage, short8 (&a)[KS][FM], short8 (&b)[KS][FN]) {
      const bf16_t* As = lds + stage * G::STAGE;
      const bf16_t* Bs = As + 256 * BK;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
        for (int j = 0; j < FN; ++j)
          b[ks][j] = *reinterpret_cast<const short8*>(Bs + swz<BK>(wn * WTN + 16 * j + fr,
                                                                   ks * 4 + fq));
#pragma unroll
        for (int i = 0; i < FM; ++i)
          a[ks][i] = *reinterpret_cast<const short8*>(As + swz<BK>(wm * WTM + 16 * i + fr,
                                                                   ks * 4 + fq));
      }
    };
    auto mma = [&](const short8 (&a)[KS][FM], const short8 (&b)[KS][FN]) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(a[ks][i], b[ks][j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    };
    // step t: stage t's fragments are in `ca/cb`; wait for stage t+1, refill stage
    // t's buffer with stage t+NS, read stage t+1 into `na/nb`, MFMAs on stage t
    auto step = [&](int t, short8 (&ca)[KS][FM], short8 (&cb)[KS][FN], short8 (&na)[KS][FM],
                    short8 (&nb)[KS][FN]) {
      if (t + 1 < n_loc) {
        wait_vm<(NS - 2) * L>();                            // stage t+1 landed
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // stage t is in registers
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        const int nxt = t + NS;
        issue(t % NS, nxt < klast ? nxt : klast);
        ldfrag((t + 1) % NS, na, nb);
      }
      mma(ca, cb);
      __builtin_amdgcn_sched_barrier(0);
    };
#pragma unroll
    for (int st = 0; st < NS; ++st) issue(st, st < klast ? st : klast);
    wait_vm<(NS - 1) * L>();
    __builtin_amdgcn_s_barrier();
    short8 a0[KS][FM], b0[KS][FN], a1[KS][FM], b1[KS][FN];
    ldfrag(0, a0, b0);
    for (int t = 0; t < n_loc; t += 2) {
      step(t, a0, b0, a1, b1);
      if (t + 1 < n_loc) step(t + 1, a1, b1, a0, b0);
    }
  } else {
    // ---- pipeline: stages 0..NS-2 in flight before the loop; step t waits for its
    // own stage (NS-2 younger stages stay outstanding), passes ONE raw barrier (every
    // wave's DMA for stage t has landed, and every wave is done reading stage t-1's
    // buffer), refills that buffer with stage t+NS-1, then computes stage t.  Past
    // the slice end the refill re-reads the last stage into a buffer nobody reads,
    // which keeps the vmcnt count constant (branch-free pipeline).
#pragma unroll
    for (int s = 0; s < NS - 1; ++s) issue(s, s < klast ? s : klast);
    for (int t0 = 0; t0 < n_loc; t0 += NS) {
#pragma unroll
      for (int u = 0; u < NS; ++u) {
        const int t = t0 + u;
        if (t < n_loc) {
          wait_vm<(NS - 2) * L>();
          __builtin_amdgcn_s_barrier();
          __builtin_amdgcn_sched_barrier(0);
          const int nxt = t + NS - 1;
          issue((u + NS - 1) % NS, nxt < klast ? nxt : klast);
          compute(u);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  }
  wait_vm<0>();

  // ---- epilogue: lane holds rows wm*WTM + 16i + 4fq + r, tile columns wn*WTN + 16j + fr
  if (MODE == 2 || MODE == 3) {
    // MODE 3: fp16 slabs (one K-slice's fp32 sum rounded to 11 bits)
    using P = std::conditional_t<MODE == 2, float, _Float16>;
    P* o = reinterpret_cast<P*>(out) + (int64_t)split * M * N + (int64_t)m0 * N +
           (int64_t)tile * BN + wn * WTN + fr;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * WTM + 16 * i + 4 * fq + r;
        if (row < Mt) {
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            float v = acc[i][j][r];
            // fp16 slabs saturate at +-65504: an out-of-range partial stays finite
            if constexpr (MODE == 3) v = fminf(fmaxf(v, -65504.f), 65504.f);
            o[(int64_t)row * N + 16 * j] = (P)v;
          }
        }
      }
  } else if (MODE == 0) {
    bf16_t* o = reinterpret_cast<bf16_t*>(out) + (int64_t)m0 * ldo + (int64_t)tile * BN +
                wn * WTN + fr;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * WTM + 16 * i + 4 * fq + r;
        if (row < Mt) {
#pragma unroll
          for (int j = 0; j < FN; ++j) o[(int64_t)row * ldo + 16 * j] = f2bf(acc[i][j][r]);
        }
      }
  } else {
    bf16_t* o = reinterpret_cast<bf16_t*>(out) + (int64_t)m0 * ldo + (int64_t)tile * (BN / 2) +
                wn * (WTN / 2) + fr;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * WTM + 16 * i + 4 * fq + r;
        if (row < Mt) {
#pragma unroll
          for (int j = 0; j < FN / 2; ++j)
            o[(int64_t)row * ldo + 16 * j] = f2bf(silu(acc[i][j][r]) * acc[i][j + FN / 2][r]);
        }
      }
  }
}

// wnt bit 0: non-temporal W loads; bit 1: 32-k stages (BN >= 128); bit 2:
// register-pipelined fragment reads (BN <= 128, 64-k stages); bit 3: W is
// tile-packed for this bn / mode (ops.tgemm_pack; 64-k stages)
template <int BN, int MODE>
int launch_bn(void* out, const bf16_t* X, const bf16_t* W, int M, int N, int K, int S, int ldo,
              int wnt, hipStream_t s) {
  const int ntiles = MODE == 1 ? N / (BN / 2) : N / BN;
  const dim3 grid(ntiles * S * ((M + 255) / 256)), block(512);
  const bool nt = wnt & 1, bk32 = wnt & 2, pipe = wnt & 4, pk = wnt & 8;
  if (bk32 && pipe) return -22;
  if (pk) {  // tile-packed W: 64-k stages, shared or register-pipelined ring
    if (bk32) return -25;
    if constexpr (BN <= 128) {
      if (pipe) {
        if (nt)
          tgemm_kernel<BN, MODE, 1, 64, 1, 1><<<grid, block, 0, s>>>(out, X, W, M, N, K, S, ldo);
        else
          tgemm_kernel<BN, MODE, 0, 64, 1, 1><<<grid, block, 0, s>>>(out, X, W, M, N, K, S, ldo);
        return (int)hipGetLastError();
      }
    } else {
      if (pipe) return -23;
    }
    if (nt)
      tgemm_kernel<BN, MODE, 1, 64, 0, 1><<<grid, block, 0, s>>>(out, X, W, M, N, K, S, ldo);
    else
      tgemm_kernel<BN, MODE, 0, 64, 0, 1><<<grid, block, 0, s>>>(out, X, W, M, N, K, S, ldo);
    return (int)hipGetLastError();
  }
  if constexpr (BN >= 128) {
    if (bk32) {
      if (nt)
        tgemm_kernel<BN, MODE, 1, 32, 0><<<grid, block, 0, s>>>(out, X, W, M, N, K, S, ldo);
      else
        tgemm_kernel<BN, MODE, 0, 32, 0><<<grid, block, 0, s>>>(out, X, W, M, N, K, S, ldo);
      return (int)hipGetLastError();
    }
  } else {
    if (bk32) return -21;
  }
  if constexpr (BN <= 128) {
    if (pipe) {
      if (nt)
        tgemm_kernel<BN, MODE, 1, 64, 1><<<grid, block, 0, s>>>(out, X, W, M, N, K, S, ldo);
      else
        tgemm_kernel<BN, MODE, 0, 64, 1><<<grid, block, 0, s>>>(out, X, W, M, N, K, S, ldo);
      return (int)hipGetLastError();
    }
  } else {
    if (pipe) return -23;
  }
  if (nt)
    tgemm_kernel<BN, MODE, 1, 64, 0><<<grid, block, 0, s>>>(out, X, W, M, N, K, S, ldo);
  else
    tgemm_kernel<BN, MODE, 0, 64, 0><<<grid, block, 0, s>>>(out, X, W, M, N, K, S, ldo);
  return (int)hipGetLastError();
}

template <int MODE>
int launch_mode(void* out, const bf16_t* X, const bf16_t* W, int M, int N, int K, int S, int ldo,
                int bn, int wnt, hipStream_t s) {
  if (bn == 64) return launch_bn<64, MODE>(out, X, W, M, N, K, S, ldo, wnt, s);
  if (bn == 128) return launch_bn<128, MODE>(out, X, W, M, N, K, S, ldo, wnt, s);
  if (bn == 256) return launch_bn<256, MODE>(out, X, W, M, N, K, S, ldo, wnt, s);
  return -20;
}

}  // namespace

extern "C" {

// Returns 0 on success, < 0 for a shape the kernel does not cover (checked
// BEFORE any launch).  mode 0: bf16 out[M, ldo]; mode 1: SwiGLU bf16 out[M, ldo]
// from W = [Wg; Wu] ([2N, K]); mode 2: fp32 slabs out[S][M][N].
int omnia_tgemm(int mode, void* out, const void* X, const void* W, int M, int N, int K, int S,
                int bn, int wnt, int ldo, hipStream_t s) {
  if (mode < 0 || mode > 3) return -1;
  if (M < 1 || (int64_t)((M + 255) / 256) * S * (N / 64) > (1 << 30)) return -2;
  if (K % 64 || K <= 0) return -3;
  if (S < 1 || S > 16 || S > K / 64) return -4;
  if (bn != 64 && bn != 128 && bn != 256) return -5;
  const int cols = mode == 1 ? bn / 2 : bn;
  if (N % cols) return -6;
  if (mode < 2 && S != 1) return -7;
  if ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W) |
       reinterpret_cast<uintptr_t>(out)) & 15)
    return -8;
  if (mode < 2 && ldo < N) return -9;
  const bf16_t* x = (const bf16_t*)X;
  const bf16_t* w = (const bf16_t*)W;
  if (mode == 0) return launch_mode<0>(out, x, w, M, N, K, S, ldo, bn, wnt, s);
  if (mode == 1) return launch_mode<1>(out, x, w, M, N, K, S, ldo, bn, wnt, s);
  if (mode == 2) return launch_mode<2>(out, x, w, M, N, K, S, N, bn, wnt, s);
  return launch_mode<3>(out, x, w, M, N, K, S, N, bn, wnt, s);
}

}  // extern "C"
