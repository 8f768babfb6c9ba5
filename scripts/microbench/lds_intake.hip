// Per-CU operand intake microbenchmark for the M = 256 decode GEMM shape
// (tgemm.hip): every block streams the shared 256 x K activation slab ("x",
// L2-resident, re-read by every block) and its own 128 x K weight rows ("W",
// HBM) in 64-k stages through a 3-deep LDS ring with counted waits -- the
// tgemm staging pipeline without the MFMAs.  Modes:
//   0  x by LDS-DMA, W by LDS-DMA          (tgemm today)
//   1  x by LDS-DMA, W by global_load_dwordx4 into registers (+ ds_write)
//   2  W by LDS-DMA alone
//   3  x by LDS-DMA alone
//   4  W by register loads alone
// Question: do the L2-hot x requests and the HBM W requests share one per-CU
// queue (times add) when both use LDS-DMA, and does moving W to plain loads
// let them overlap?
//   hipcc --offload-arch=gfx950 -O3 -o lds_intake lds_intake.hip && ./lds_intake
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef short short8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory"); }

constexpr int BK = 64, BM = 256, BN = 128, NS = 3;
constexpr int XST = BM * BK, WST = BN * BK, STAGE = XST + WST;  // bf16 elements

template <int MODE>
__global__ __launch_bounds__(512, 1) void intake(const uint16_t* __restrict__ X,
                                                 const uint16_t* __restrict__ W, int K,
                                                 int* __restrict__ sink) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[NS * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nk = K / BK;
  // 8 rows x 128 B per wave instruction: lane -> row lane/8, chunk lane%8
  const int lr = lane >> 3, lc = lane & 7;
  const uint16_t* xs[4];
  for (int i = 0; i < 4; ++i) xs[i] = X + (int64_t)(8 * (w * 4 + i) + lr) * K + lc * 8;
  const uint16_t* ws[2];
  for (int i = 0; i < 2; ++i)
    ws[i] = W + ((int64_t)blockIdx.x * BN + 8 * (w * 2 + i) + lr) * K + lc * 8;
  const int xd = (8 * w * 4) * BK, wd = XST + (8 * w * 2) * BK;
  constexpr bool XON = MODE != 2 && MODE != 4, WDMA = MODE == 0 || MODE == 2,
                 WREG = MODE == 1 || MODE == 4;
  short8 wr[NS][2];
  short8 acc = {0, 0, 0, 0, 0, 0, 0, 0};
  auto issue = [&](int st, int kl) {
    uint16_t* base = lds + st * STAGE;
    if (XON)
      for (int i = 0; i < 4; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(xs[i] + kl * BK),
                                         (lds_ptr_t)(base + xd + i * 512), 16, 0, 0);
    if (WDMA)
      for (int i = 0; i < 2; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(ws[i] + kl * BK),
                                         (lds_ptr_t)(base + wd + i * 512), 16, 0, 0);
  };
  auto wload = [&](int r, int kl) {
    if (WREG)
      for (int i = 0; i < 2; ++i) wr[r][i] = *reinterpret_cast<const short8*>(ws[i] + kl * BK);
  };
  const int klast = nk - 1;
  for (int s = 0; s < NS - 1; ++s) {
    issue(s, s);
    wload(s, s);
  }
  constexpr int L = (XON ? 4 : 0) + (WDMA || WREG ? 2 : 0);
  for (int t0 = 0; t0 < nk; t0 += NS) {
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      const int t = t0 + u;
      if (t < nk) {
        wait_vm<(NS - 2) * L>();
        __builtin_amdgcn_s_barrier();
        const int nx = t + NS - 1 < klast ? t + NS - 1 : klast;
        issue((u + NS - 1) % NS, nx);
        wload((u + NS - 1) % NS, nx);
        if (WREG) {  // consume stage t's W registers: write them into the stage (as tgemm would)
          uint16_t* base = lds + u * STAGE;
          for (int i = 0; i < 2; ++i)
            *reinterpret_cast<short8*>(base + wd + i * 512 + lane * 8) = wr[u][i];
        }
        // touch the stage so the loads are live
        acc += *reinterpret_cast<const short8*>(lds + u * STAGE + (tid & 511) * 8);
      }
    }
  }
  wait_vm<0>();
  if (acc[0] == (short)0x1234 && acc[1] == (short)0x4321) sink[0] = 1;
}

int main() {
  const int K = 4096, nblk_list[] = {224, 256};
  const size_t xbytes = (size_t)BM * K * 2;
  std::vector<uint16_t*> Ws;
  const size_t wrows = 256 * BN;  // rows for 256 blocks
  const size_t wbytes = wrows * K * 2;  // 256 MB
  uint16_t* X;
  int* sink;
  hipMalloc(&X, xbytes);
  hipMalloc(&sink, 4);
  hipMemset(X, 1, xbytes);
  for (int c = 0; c < 4; ++c) {  // rotate 4 weight copies: > the 256 MB MALL
    uint16_t* W;
    hipMalloc(&W, wbytes);
    hipMemset(W, 2, wbytes);
    Ws.push_back(W);
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"x dma + W dma", "x dma + W regs", "W dma only", "x dma only",
                         "W regs only"};
  for (int nb : nblk_list) {
    for (int mode = 0; mode < 5; ++mode) {
      auto launch = [&](int i) {
        const uint16_t* W = Ws[i % 4];
        switch (mode) {
          case 0: intake<0><<<nb, 512>>>(X, W, K, sink); break;
          case 1: intake<1><<<nb, 512>>>(X, W, K, sink); break;
          case 2: intake<2><<<nb, 512>>>(X, W, K, sink); break;
          case 3: intake<3><<<nb, 512>>>(X, W, K, sink); break;
          default: intake<4><<<nb, 512>>>(X, W, K, sink); break;
        }
      };
      for (int i = 0; i < 8; ++i) launch(i);
      hipDeviceSynchronize();
      const int iters = 40;
      hipEventRecord(e0);
      for (int i = 0; i < iters; ++i) launch(i);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 1000 / iters;
      const double wmb = (mode == 3) ? 0 : nb * (double)BN * K * 2 / 1e6;
      const double xmb = (mode == 2 || mode == 4) ? 0 : nb * (double)xbytes / 1e6;
      printf("blocks %3d  %-16s %7.1f us  W %6.0f MB -> %5.2f TB/s   x(L2) %6.0f MB -> %5.2f TB/s\n",
             nb, names[mode], us, wmb, wmb / us / 1e6, xmb, xmb / us / 1e6);
      fflush(stdout);
    }
  }
  return 0;
}
