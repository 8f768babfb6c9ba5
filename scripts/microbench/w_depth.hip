// Weight-stream depth microbenchmark (the tgemm staging shape without MFMAs):
// 224 / 256 blocks x 512 threads, one block per CU; each block streams its own
// 128 weight rows x K = 4096 (bf16, 1 MiB) in 64-k stages of 16 KiB by LDS-DMA
// through an NSW-deep LDS ring (static stage indices, counted vmcnt, one raw
// barrier per stage), optionally alongside the 256-row activation slab (L2-hot,
// NSX-deep ring) that tgemm re-reads per block.  Prints the weight stream rate
// against the ring depth: is the M = 256 decode GEMM latency-bound on the
// weight bytes in flight per CU?
//   hipcc --offload-arch=gfx950 -O3 -o w_depth w_depth.hip && ./w_depth
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef short short8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;
template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory"); }

constexpr int BK = 64, BN = 128, BM = 256;
constexpr int WST = BN * BK, XST = BM * BK;  // elements

// NSX == 0: weights only.  Stage s of W lives in slot s % NSW, of x in s % NSX;
// the loop is unrolled by NSW * max(NSX,1) so every slot index is static.
template <int NSW, int NSX, int PACK = 0>
__global__ __launch_bounds__(512, 1) void stream(const uint16_t* __restrict__ X,
                                                 const uint16_t* __restrict__ W, int K,
                                                 int* __restrict__ sink) {
  __shared__ __attribute__((aligned(16))) uint16_t wl[NSW * WST];
  __shared__ __attribute__((aligned(16))) uint16_t xl[(NSX ? NSX : 1) * XST];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane >> 3, lc = lane & 7;
  const uint16_t* ws[2];
  for (int i = 0; i < 2; ++i)
    ws[i] = PACK ? W + (int64_t)blockIdx.x * BN * K + (8 * (w * 2 + i) + lr) * BK + lc * 8
                 : W + ((int64_t)blockIdx.x * BN + 8 * (w * 2 + i) + lr) * K + lc * 8;
  // PACK: the block's weights stored stage-major ([block][k-stage][128 rows][64]),
  // so each 16 KiB stage is one contiguous run instead of 128 B from 128 rows
  const uint16_t* xs[4];
  for (int i = 0; i < 4; ++i) xs[i] = X + (int64_t)(8 * (w * 4 + i) + lr) * K + lc * 8;
  const int nk = K / BK, klast = nk - 1;
  auto wissue = [&](int slot, int kl) {
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(ws[i] + kl * (PACK ? BN * BK : BK)),
                                       (lds_ptr_t)(wl + slot * WST + (w * 2 + i) * 512), 16, 0, 0);
  };
  auto xissue = [&](int slot, int kl) {
    if (NSX)
      for (int i = 0; i < 4; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(xs[i] + kl * BK),
                                         (lds_ptr_t)(xl + slot * XST + (w * 4 + i) * 512), 16, 0,
                                         0);
  };
  // issue order per step s: x(s + NSX - 1), then W(s + NSW - 1); prologue as
  // virtual steps.  NSW >= NSX: W(t) is older than x(t), so waiting for x(t)
  // (or for W(t) when NSX == 0) covers both.
  constexpr int LW = 2, LX = NSX ? 4 : 0, L = LW + LX;
  constexpr int WAITN = NSX ? LW + (NSX - 2) * L : (NSW - 2) * LW;
  static_assert(NSX == 0 || NSW >= NSX, "W ring at least as deep");
  constexpr int U = NSW * (NSX ? NSX : 1);
#pragma unroll
  for (int j = -(NSW - 1); j < 0; ++j) {
    if (NSX && j + NSX - 1 >= 0) xissue(j + NSX - 1, j + NSX - 1);
    wissue(j + NSW - 1, j + NSW - 1 < klast ? j + NSW - 1 : klast);
  }
  short8 acc = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int t0 = 0; t0 < nk; t0 += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = t0 + u;
      if (t < nk) {
        wait_vm<WAITN>();
        __builtin_amdgcn_s_barrier();
        const int nx = t + NSX - 1, nw = t + NSW - 1;
        if (NSX) xissue((u + NSX - 1) % (NSX ? NSX : 1), nx < klast ? nx : klast);
        wissue((u + NSW - 1) % NSW, nw < klast ? nw : klast);
      }
    }
  }
  wait_vm<0>();
  __syncthreads();
  acc += *reinterpret_cast<const short8*>(wl + tid * 8 % WST);
  if (NSX) acc += *reinterpret_cast<const short8*>(xl + tid * 8);
  if (acc[0] == (short)0x1234 && acc[1] == (short)0x4321) sink[0] = 1;
}

int main() {
  const int K = 4096;
  const size_t wbytes = (size_t)256 * BN * K * 2, xbytes = (size_t)BM * K * 2;
  std::vector<uint16_t*> Ws;
  uint16_t* X;
  int* sink;
  (void)hipMalloc(&X, xbytes);
  (void)hipMalloc(&sink, 4);
  (void)hipMemset(X, 1, xbytes);
  for (int c = 0; c < 4; ++c) {
    uint16_t* W;
    (void)hipMalloc(&W, wbytes);
    (void)hipMemset(W, 2, wbytes);
    Ws.push_back(W);
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  struct Cfg { int nsw, nsx, pack; void (*k)(const uint16_t*, const uint16_t*, int, int*); };
  Cfg cfgs[] = {{3, 0, 0, stream<3, 0>}, {3, 0, 1, stream<3, 0, 1>}, {4, 0, 1, stream<4, 0, 1>},
                {6, 0, 1, stream<6, 0, 1>}, {3, 3, 0, stream<3, 3>}, {3, 3, 1, stream<3, 3, 1>},
                {4, 3, 1, stream<4, 3, 1>}};
  for (int nb : {224, 256}) {
    for (const Cfg& c : cfgs) {
      auto launch = [&](int i) { c.k<<<nb, 512>>>(X, Ws[i % 4], K, sink); };
      for (int i = 0; i < 8; ++i) launch(i);
      (void)hipDeviceSynchronize();
      const int iters = 40;
      (void)hipEventRecord(e0);
      for (int i = 0; i < iters; ++i) launch(i);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 1000 / iters;
      const double wmb = nb * (double)BN * K * 2 / 1e6;
      printf("blocks %3d  W ring %d (%2d KiB in flight) %s  x ring %d: %6.1f us  W %.2f TB/s\n", nb,
             c.nsw, (c.nsw - 1) * 16, c.pack ? "packed " : "rowmajor", c.nsx, us, wmb / us);
      fflush(stdout);
    }
  }
  return 0;
}
