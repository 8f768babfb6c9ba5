// One-shot intra-node all-reduce over xGMI peer memory.
//
// Decode-step tensor-parallel all-reduces are tiny (B x d x 2 B = 16 KiB per
// sequence at d = 8192) and latency-bound, so instead of a ring (one xGMI link
// per step) every rank reads all peers' buffers DIRECTLY over the fully
// connected xGMI mesh and reduces locally: one hop, all 7 links busy at once.
//
// Protocol (one launch, graph-capturable, no host involvement):
//   * every rank owns an IPC-exported region: 2 data slots (epoch parity) of
//     `slot_bytes` each + a flag array flags[block][peer];
//   * block b copies ITS slice of the input into data[epoch & 1] of its own
//     region, then (system-scope release) stores `epoch` into flags[b][me] of
//     EVERY peer's region;
//   * block b waits (bounded spin, system-scope acquire) until its own
//     flags[b][p] == epoch for all p, then sums slice b of every peer's slot
//     in rank order (deterministic, identical on all ranks) into the output;
//   * the epoch lives in device memory per block (read at start, bumped at the
//     end) so a captured hipGraph replays correctly.
// Slot reuse is safe with 2 parity slots: a rank overwrites slot e&1 in call
// e+2 only after every peer has signalled call e+1, i.e. finished reading e.
// Every spin is bounded; a timeout sets err[0] and the kernel exits (the host
// raises) instead of hanging the GPU.
#include <string.h>

#include "common.h"

using namespace omnia;

namespace {

constexpr int kMaxRanks = 8;
constexpr int kBlocks = 32;  // slices; flags[kBlocks][kMaxRanks]

struct PeerPtrs {
  char* data[kMaxRanks];   // base of each rank's region (data slots at offset 0)
  int* flags[kMaxRanks];   // each rank's flag array
};

__device__ __forceinline__ void st_release_sys(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ int ld_acquire_sys(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void ar_oneshot_kernel(bf16_t* __restrict__ out,
                                                         const bf16_t* __restrict__ in,
                                                         PeerPtrs peers, int* __restrict__ epochs,
                                                         int* __restrict__ err, int64_t n,
                                                         int64_t slot_bytes, int rank, int world) {
  const int b = blockIdx.x, tid = threadIdx.x;
  __shared__ int s_epoch;
  if (tid == 0) s_epoch = epochs[b] + 1;
  __syncthreads();
  const int epoch = s_epoch;
  const int64_t slot = (epoch & 1) * slot_bytes;
  // slice of 16-B vectors owned by this block
  const int64_t nv = n / 8;
  const int64_t per = (nv + kBlocks - 1) / kBlocks;
  const int64_t v0 = b * per, v1 = v0 + per < nv ? v0 + per : nv;

  // 1. stage my slice into my own exported slot
  uint4v* mine = reinterpret_cast<uint4v*>(peers.data[rank] + slot);
  const uint4v* src = reinterpret_cast<const uint4v*>(in);
  for (int64_t v = v0 + tid; v < v1; v += 256) mine[v] = src[v];
  __syncthreads();
  // 2. publish: release at system scope, then flag every peer
  if (tid < world) {
    __threadfence_system();
    st_release_sys(peers.flags[tid] + b * kMaxRanks + rank, epoch);
  }
  // 3. wait for every peer's slice b (bounded)
  if (tid < world) {
    const int* f = peers.flags[rank] + b * kMaxRanks + tid;
    long spins = 0;
    while (ld_acquire_sys(f) < epoch) {
      if (++spins > (1L << 26)) {
        atomicExch(err, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  // 4. reduce slice b across ranks in rank order (fp32 accumulate)
  for (int64_t v = v0 + tid; v < v1; v += 256) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int p = 0; p < world; ++p) {
      const uint4v x = __builtin_nontemporal_load(
          reinterpret_cast<const uint4v*>(peers.data[p] + slot) + v);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc[2 * q] += bf2f((uint16_t)(x[q] & 0xffffu));
        acc[2 * q + 1] += bf2f((uint16_t)(x[q] >> 16));
      }
    }
    uint4v o;
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = pack_bf2(acc[2 * q], acc[2 * q + 1]);
    reinterpret_cast<uint4v*>(out)[v] = o;
  }
  __syncthreads();
  if (tid == 0) epochs[b] = epoch;
}

}  // namespace

extern "C" {

int omnia_ipc_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

// Allocates an uncached (fine-grained) region visible to peers: data slots +
// flags.  Returns 0 / hip error.
int omnia_ipc_alloc(void** ptr, int64_t bytes) {
  hipError_t e = hipExtMallocWithFlags(ptr, (size_t)bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(*ptr, 0, (size_t)bytes);
}

int omnia_ipc_free(void* ptr) { return (int)hipFree(ptr); }

int omnia_ipc_get_handle(void* ptr, void* handle_out) {
  return (int)hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(handle_out), ptr);
}

int omnia_ipc_open(const void* handle, void** ptr) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

int omnia_ipc_close(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }

int omnia_ar_blocks() { return kBlocks; }
int omnia_ar_max_ranks() { return kMaxRanks; }

// regions[p]: base pointer of rank p's region (own one from omnia_ipc_alloc,
// peers' from omnia_ipc_open).  Layout: [2 * slot_bytes data][flags int32
// kBlocks*kMaxRanks].  n = bf16 elements, multiple of 8, 2*n <= slot_bytes.
int omnia_ar_oneshot(void* out, const void* in, void* const* regions, int* epochs, int* err,
                     int64_t n, int64_t slot_bytes, int rank, int world, hipStream_t s) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world) return -1;
  if (n % 8 || 2 * n > slot_bytes || slot_bytes % 16) return -2;
  PeerPtrs pp{};
  for (int p = 0; p < world; ++p) {
    if (!regions[p]) return -3;
    pp.data[p] = reinterpret_cast<char*>(regions[p]);
    pp.flags[p] = reinterpret_cast<int*>(reinterpret_cast<char*>(regions[p]) + 2 * slot_bytes);
  }
  ar_oneshot_kernel<<<kBlocks, 256, 0, s>>>((bf16_t*)out, (const bf16_t*)in, pp, epochs, err, n,
                                            slot_bytes, rank, world);
  return (int)hipGetLastError();
}

}  // extern "C"
