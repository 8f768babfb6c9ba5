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
//
// Two-shot (reduce-scatter + all-gather) for decode messages above ~256 KiB:
// one-shot makes every rank read (world - 1) x n bytes over xGMI, two-shot reads
// 2 (world - 1) / world x n.  Rows of the [M, d] input are split into world
// chunks; rank r reduces chunk r over all peers into its own result slot, and
// every rank then gathers all chunks.  The NORM variant fuses the decoder's
// residual add + RMSNorm into the owning rank's reduce (it holds whole rows):
// residual <- bf16(sum) + residual, out <- RMSNorm(residual) * w, and gathers
// both, so a tensor-parallel layer boundary is ONE kernel.
// Region layout: [2 x slot data][2 x slot result][flags1][flags2].
#include <string.h>

#include "common.h"

using namespace omnia;

namespace {

constexpr int kMaxRanks = 8;
constexpr int kBlocks = 32;  // slices; flags[kBlocks][kMaxRanks]

struct PeerPtrs {
  char* data[kMaxRanks];   // base of each rank's region (data slots at offset 0)
  int* flags[kMaxRanks];   // each rank's phase-1 flag array
  int* flags2[kMaxRanks];  // each rank's phase-2 flag array (two-shot)
};

// bounded wait until flags[b][p] >= epoch for every peer p (threads tid < world)
__device__ __forceinline__ void wait_peers(int* const* flags, int b, int rank, int world,
                                           int epoch, int* err) {
  const int tid = threadIdx.x;
  if (tid < world) {
    const int* f = flags[rank] + b * kMaxRanks + tid;
    long spins = 0;
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      if (++spins > (1L << 26)) {
        atomicExch(err, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

__device__ __forceinline__ void publish(int* const* flags, int b, int rank, int world,
                                        int epoch) {
  __syncthreads();
  if ((int)threadIdx.x < world) {
    __threadfence_system();
    __hip_atomic_store(flags[threadIdx.x] + b * kMaxRanks + rank, epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

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

// All-gather of an opaque byte buffer (nbytes per rank, multiple of 16) into
// out[world][nbytes]: block b stages its slice of `in` into my data slot,
// publishes, waits for every peer's slice b, then copies slice b of every peer's
// slot into out[p].  Same flags / epochs / parity slots as the one-shot
// all-reduce (every collective of a group bumps every block's epoch once).
__global__ __launch_bounds__(256) void ar_allgather_kernel(char* __restrict__ out,
                                                           const char* __restrict__ in,
                                                           PeerPtrs peers, int* __restrict__ epochs,
                                                           int* __restrict__ err, int64_t nbytes,
                                                           int64_t slot_bytes, int rank, int world) {
  const int b = blockIdx.x, tid = threadIdx.x;
  __shared__ int s_epoch;
  if (tid == 0) s_epoch = epochs[b] + 1;
  __syncthreads();
  const int epoch = s_epoch;
  const int64_t slot = (epoch & 1) * slot_bytes;
  const int64_t nv = nbytes / 16;
  const int64_t per = (nv + kBlocks - 1) / kBlocks;
  const int64_t v0 = b * per, v1 = v0 + per < nv ? v0 + per : nv;
  uint4v* mine = reinterpret_cast<uint4v*>(peers.data[rank] + slot);
  const uint4v* src = reinterpret_cast<const uint4v*>(in);
  for (int64_t v = v0 + tid; v < v1; v += 256) mine[v] = src[v];
  publish(peers.flags, b, rank, world, epoch);
  wait_peers(peers.flags, b, rank, world, epoch, err);
  for (int p = 0; p < world; ++p) {
    const uint4v* ps = reinterpret_cast<const uint4v*>(peers.data[p] + slot);
    uint4v* dst = reinterpret_cast<uint4v*>(out + (int64_t)p * nbytes);
    for (int64_t v = v0 + tid; v < v1; v += 256) dst[v] = __builtin_nontemporal_load(ps + v);
  }
  __syncthreads();
  if (tid == 0) epochs[b] = epoch;
}

// All-to-all of an opaque byte buffer: in = [world][chunk] (chunk bytes for each
// destination rank, multiple of 16), out = [world][chunk] (chunk p = what rank p
// sent to me).  Block b stages slice b of every destination chunk into my data
// slot, publishes, waits for every peer's slice b, then pulls slice b of MY
// chunk out of every peer's slot (peer p's slot holds its whole send buffer, so
// my chunk sits at offset rank * chunk) -- one hop over the xGMI mesh per pair,
// all links busy at once.  Same flags / epochs / parity slots as the other
// collectives of the group (the EP all-to-all of DP-attention + EP, K15).
__global__ __launch_bounds__(256) void ar_alltoall_kernel(char* __restrict__ out,
                                                          const char* __restrict__ in,
                                                          PeerPtrs peers, int* __restrict__ epochs,
                                                          int* __restrict__ err, int64_t chunk,
                                                          int64_t slot_bytes, int rank, int world) {
  const int b = blockIdx.x, tid = threadIdx.x;
  __shared__ int s_epoch;
  if (tid == 0) s_epoch = epochs[b] + 1;
  __syncthreads();
  const int epoch = s_epoch;
  const int64_t slot = (epoch & 1) * slot_bytes;
  const int64_t nv = chunk / 16;
  const int64_t per = (nv + kBlocks - 1) / kBlocks;
  const int64_t v0 = b * per, v1 = v0 + per < nv ? v0 + per : nv;
  uint4v* mine = reinterpret_cast<uint4v*>(peers.data[rank] + slot);
  const uint4v* src = reinterpret_cast<const uint4v*>(in);
  for (int q = 0; q < world; ++q)
    for (int64_t v = v0 + tid; v < v1; v += 256) mine[q * nv + v] = src[q * nv + v];
  publish(peers.flags, b, rank, world, epoch);
  wait_peers(peers.flags, b, rank, world, epoch, err);
  for (int p = 0; p < world; ++p) {
    const uint4v* ps = reinterpret_cast<const uint4v*>(peers.data[p] + slot) + rank * nv;
    uint4v* dst = reinterpret_cast<uint4v*>(out) + p * nv;
    for (int64_t v = v0 + tid; v < v1; v += 256) dst[v] = __builtin_nontemporal_load(ps + v);
  }
  __syncthreads();
  if (tid == 0) epochs[b] = epoch;
}

// Point-to-point exchange (one ring hop of context-parallel attention): every
// rank publishes `in` (nbytes) and receives rank `src`'s into `out`.  It waits on
// every peer's flag (not only src's): that is what makes the parity-slot reuse
// safe -- a slot is rewritten two calls later only after every reader of it has
// signalled the next call.
__global__ __launch_bounds__(256) void ar_sendrecv_kernel(char* __restrict__ out,
                                                          const char* __restrict__ in,
                                                          PeerPtrs peers, int* __restrict__ epochs,
                                                          int* __restrict__ err, int64_t nbytes,
                                                          int64_t slot_bytes, int rank, int world,
                                                          int src_rank) {
  const int b = blockIdx.x, tid = threadIdx.x;
  __shared__ int s_epoch;
  if (tid == 0) s_epoch = epochs[b] + 1;
  __syncthreads();
  const int epoch = s_epoch;
  const int64_t slot = (epoch & 1) * slot_bytes;
  const int64_t nv = nbytes / 16;
  const int64_t per = (nv + kBlocks - 1) / kBlocks;
  const int64_t v0 = b * per, v1 = v0 + per < nv ? v0 + per : nv;
  uint4v* mine = reinterpret_cast<uint4v*>(peers.data[rank] + slot);
  const uint4v* src = reinterpret_cast<const uint4v*>(in);
  for (int64_t v = v0 + tid; v < v1; v += 256) mine[v] = src[v];
  publish(peers.flags, b, rank, world, epoch);
  wait_peers(peers.flags, b, rank, world, epoch, err);
  const uint4v* ps = reinterpret_cast<const uint4v*>(peers.data[src_rank] + slot);
  uint4v* dst = reinterpret_cast<uint4v*>(out);
  for (int64_t v = v0 + tid; v < v1; v += 256) dst[v] = __builtin_nontemporal_load(ps + v);
  __syncthreads();
  if (tid == 0) epochs[b] = epoch;
}

// Row chunk of (rank r, block b): [r*R + b*Rb, min(r*R + (b+1)*Rb, (r+1)*R, M)).
// VEC = 16-B vectors per thread per row (d <= 256 * 8 * VEC).
template <bool NORM, int VEC>
__global__ __launch_bounds__(256) void ar_twoshot_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ in, bf16_t* __restrict__ residual,
    const bf16_t* __restrict__ w, PeerPtrs peers, int* __restrict__ epochs,
    int* __restrict__ err, int M, int d, int64_t slot_bytes, int rank, int world, float eps) {
  __shared__ float scratch[8];
  __shared__ int s_epoch;
  const int b = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) s_epoch = epochs[b] + 1;
  __syncthreads();
  const int epoch = s_epoch;
  const int64_t dslot = (epoch & 1) * slot_bytes, rslot = 2 * slot_bytes + dslot;
  const int R = (M + world - 1) / world, Rb = (R + kBlocks - 1) / kBlocks;
  const int dv = d / 8;  // 16-B vectors per row
  auto rows = [&](int r, int& lo, int& hi) {
    lo = r * R + b * Rb;
    hi = min(min(lo + Rb, (r + 1) * R), M);
  };
  // 1. stage rows (r, b) of every chunk into my data slot
  uint4v* mine = reinterpret_cast<uint4v*>(peers.data[rank] + dslot);
  const uint4v* src = reinterpret_cast<const uint4v*>(in);
  for (int r = 0; r < world; ++r) {
    int lo, hi;
    rows(r, lo, hi);
    for (int64_t v = (int64_t)lo * dv + tid; v < (int64_t)hi * dv; v += 256) mine[v] = src[v];
  }
  publish(peers.flags, b, rank, world, epoch);
  wait_peers(peers.flags, b, rank, world, epoch, err);
  // 2. reduce my rows over all peers (rank order: identical on every rank)
  {
    int lo, hi;
    rows(rank, lo, hi);
    uint4v* res = reinterpret_cast<uint4v*>(peers.data[rank] + rslot);
    uint4v* res_r = res + (int64_t)M * dv;  // NORM: new residual rows after the outputs
    for (int row = lo; row < hi; ++row) {
      float acc[VEC][8];
#pragma unroll
      for (int i = 0; i < VEC; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = 0.f;
      for (int p = 0; p < world; ++p) {
        const uint4v* pd = reinterpret_cast<const uint4v*>(peers.data[p] + dslot) +
                           (int64_t)row * dv;
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          const int c = i * 256 + tid;
          if (c < dv) {
            const uint4v x = __builtin_nontemporal_load(pd + c);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              acc[i][2 * q] += bf2f((uint16_t)(x[q] & 0xffffu));
              acc[i][2 * q + 1] += bf2f((uint16_t)(x[q] >> 16));
            }
          }
        }
      }
      if (!NORM) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          const int c = i * 256 + tid;
          if (c < dv) {
            uint4v o;
#pragma unroll
            for (int q = 0; q < 4; ++q) o[q] = pack_bf2(acc[i][2 * q], acc[i][2 * q + 1]);
            res[(int64_t)row * dv + c] = o;
          }
        }
      } else {
        float ss = 0.f;
        const uint4v* rr = reinterpret_cast<const uint4v*>(residual) + (int64_t)row * dv;
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          const int c = i * 256 + tid;
          if (c < dv) {
            const uint4v r0 = rr[c];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const float a = bf2f(f2bf(acc[i][2 * q])) + bf2f((uint16_t)(r0[q] & 0xffffu));
              const float e = bf2f(f2bf(acc[i][2 * q + 1])) + bf2f((uint16_t)(r0[q] >> 16));
              acc[i][2 * q] = bf2f(f2bf(a));
              acc[i][2 * q + 1] = bf2f(f2bf(e));
              ss += acc[i][2 * q] * acc[i][2 * q] + acc[i][2 * q + 1] * acc[i][2 * q + 1];
            }
          }
        }
        ss = block_sum(ss, scratch);
        const float inv = rsqrtf(ss / (float)d + eps);
        const uint4v* wv = reinterpret_cast<const uint4v*>(w);
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          const int c = i * 256 + tid;
          if (c < dv) {
            const uint4v wq = wv[c];
            uint4v o, nr;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              o[q] = pack_bf2(acc[i][2 * q] * inv * bf2f((uint16_t)(wq[q] & 0xffffu)),
                              acc[i][2 * q + 1] * inv * bf2f((uint16_t)(wq[q] >> 16)));
              nr[q] = pack_bf2(acc[i][2 * q], acc[i][2 * q + 1]);
            }
            res[(int64_t)row * dv + c] = o;
            res_r[(int64_t)row * dv + c] = nr;
          }
        }
      }
    }
  }
  publish(peers.flags2, b, rank, world, epoch);
  wait_peers(peers.flags2, b, rank, world, epoch, err);
  // 3. gather every chunk's rows (r, b) from its owner's result slot
  uint4v* o = reinterpret_cast<uint4v*>(out);
  uint4v* nres = reinterpret_cast<uint4v*>(residual);
  for (int r = 0; r < world; ++r) {
    int lo, hi;
    rows(r, lo, hi);
    const uint4v* pr = reinterpret_cast<const uint4v*>(peers.data[r] + rslot);
    for (int64_t v = (int64_t)lo * dv + tid; v < (int64_t)hi * dv; v += 256) {
      o[v] = __builtin_nontemporal_load(pr + v);
      if (NORM) nres[v] = __builtin_nontemporal_load(pr + (int64_t)M * dv + v);
    }
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
int64_t omnia_ar_region_bytes(int64_t slot_bytes) {
  return 4 * slot_bytes + 2 * (int64_t)kBlocks * kMaxRanks * 4;
}

// Two-shot all-reduce of a row-major [M, d] bf16 tensor; with w != nullptr the
// NORM variant: residual [M, d] updated in place, out = RMSNorm(residual) * w.
// Output rows (and, NORM, the residual rows) must fit one slot.
int omnia_ar_twoshot(void* out, const void* in, void* residual, const void* w,
                     void* const* regions, int* epochs, int* err, int M, int d,
                     int64_t slot_bytes, int rank, int world, float eps, hipStream_t s) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world) return -1;
  const bool norm = w != nullptr;
  if (d % 8 || M < 1 || slot_bytes % 16) return -2;
  if ((int64_t)M * d * 2 * (norm ? 2 : 1) > slot_bytes) return -3;
  if (norm && !residual) return -4;
  PeerPtrs pp{};
  for (int p = 0; p < world; ++p) {
    if (!regions[p]) return -5;
    pp.data[p] = reinterpret_cast<char*>(regions[p]);
    pp.flags[p] = reinterpret_cast<int*>(reinterpret_cast<char*>(regions[p]) + 4 * slot_bytes);
    pp.flags2[p] = pp.flags[p] + kBlocks * kMaxRanks;
  }
  const int vec = (d / 8 + 255) / 256;
#define OMNIA_AR2(NRM, V)                                                                  \
  ar_twoshot_kernel<NRM, V><<<kBlocks, 256, 0, s>>>((bf16_t*)out, (const bf16_t*)in,        \
                                                    (bf16_t*)residual, (const bf16_t*)w, pp, \
                                                    epochs, err, M, d, slot_bytes, rank,    \
                                                    world, eps);
#define OMNIA_AR2V(V) \
  if (norm) { OMNIA_AR2(true, V) } else { OMNIA_AR2(false, V) }
  if (vec <= 1) { OMNIA_AR2V(1) }
  else if (vec <= 2) { OMNIA_AR2V(2) }
  else if (vec <= 4) { OMNIA_AR2V(4) }
  else if (vec <= 8) { OMNIA_AR2V(8) }
  else return -6;
#undef OMNIA_AR2V
#undef OMNIA_AR2
  return (int)hipGetLastError();
}
int omnia_ar_max_ranks() { return kMaxRanks; }

// out[world][nbytes] <- every rank's `in` (nbytes, multiple of 16, <= slot_bytes).
int omnia_ar_allgather(void* out, const void* in, void* const* regions, int* epochs, int* err,
                       int64_t nbytes, int64_t slot_bytes, int rank, int world, hipStream_t s) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world) return -1;
  if (nbytes % 16 || nbytes > slot_bytes || slot_bytes % 16 || nbytes <= 0) return -2;
  if ((reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(in)) & 15) return -4;
  PeerPtrs pp{};
  for (int p = 0; p < world; ++p) {
    if (!regions[p]) return -3;
    pp.data[p] = reinterpret_cast<char*>(regions[p]);
    pp.flags[p] = reinterpret_cast<int*>(reinterpret_cast<char*>(regions[p]) + 4 * slot_bytes);
    pp.flags2[p] = pp.flags[p] + kBlocks * kMaxRanks;
  }
  ar_allgather_kernel<<<kBlocks, 256, 0, s>>>((char*)out, (const char*)in, pp, epochs, err, nbytes,
                                              slot_bytes, rank, world);
  return (int)hipGetLastError();
}

static int fill_peers(PeerPtrs& pp, void* const* regions, int world, int64_t slot_bytes) {
  for (int p = 0; p < world; ++p) {
    if (!regions[p]) return -3;
    pp.data[p] = reinterpret_cast<char*>(regions[p]);
    pp.flags[p] = reinterpret_cast<int*>(reinterpret_cast<char*>(regions[p]) + 4 * slot_bytes);
    pp.flags2[p] = pp.flags[p] + kBlocks * kMaxRanks;
  }
  return 0;
}

// out[world][chunk] <- chunk `rank` of every rank's in[world][chunk]
// (world * chunk <= slot_bytes, chunk a multiple of 16).
int omnia_ar_alltoall(void* out, const void* in, void* const* regions, int* epochs, int* err,
                      int64_t chunk, int64_t slot_bytes, int rank, int world, hipStream_t s) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world) return -1;
  if (chunk % 16 || chunk <= 0 || chunk * world > slot_bytes || slot_bytes % 16) return -2;
  if ((reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(in)) & 15) return -4;
  PeerPtrs pp{};
  if (int rc = fill_peers(pp, regions, world, slot_bytes)) return rc;
  ar_alltoall_kernel<<<kBlocks, 256, 0, s>>>((char*)out, (const char*)in, pp, epochs, err, chunk,
                                             slot_bytes, rank, world);
  return (int)hipGetLastError();
}

// out[nbytes] <- rank src_rank's in[nbytes] (every rank calls with its own src).
int omnia_ar_sendrecv(void* out, const void* in, void* const* regions, int* epochs, int* err,
                      int64_t nbytes, int64_t slot_bytes, int rank, int world, int src_rank,
                      hipStream_t s) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world) return -1;
  if (src_rank < 0 || src_rank >= world) return -5;
  if (nbytes % 16 || nbytes <= 0 || nbytes > slot_bytes || slot_bytes % 16) return -2;
  if ((reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(in)) & 15) return -4;
  PeerPtrs pp{};
  if (int rc = fill_peers(pp, regions, world, slot_bytes)) return rc;
  ar_sendrecv_kernel<<<kBlocks, 256, 0, s>>>((char*)out, (const char*)in, pp, epochs, err, nbytes,
                                             slot_bytes, rank, world, src_rank);
  return (int)hipGetLastError();
}

// regions[p]: base pointer of rank p's region (own one from omnia_ipc_alloc,
// peers' from omnia_ipc_open).  Layout: [2 * slot_bytes data][2 * slot_bytes
// result][flags1 int32 kBlocks*kMaxRanks][flags2 int32 kBlocks*kMaxRanks].
// n = bf16 elements, multiple of 8, 2*n <= slot_bytes.
int omnia_ar_oneshot(void* out, const void* in, void* const* regions, int* epochs, int* err,
                     int64_t n, int64_t slot_bytes, int rank, int world, hipStream_t s) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world) return -1;
  if (n % 8 || 2 * n > slot_bytes || slot_bytes % 16) return -2;
  PeerPtrs pp{};
  for (int p = 0; p < world; ++p) {
    if (!regions[p]) return -3;
    pp.data[p] = reinterpret_cast<char*>(regions[p]);
    pp.flags[p] = reinterpret_cast<int*>(reinterpret_cast<char*>(regions[p]) + 4 * slot_bytes);
    pp.flags2[p] = pp.flags[p] + kBlocks * kMaxRanks;
  }
  ar_oneshot_kernel<<<kBlocks, 256, 0, s>>>((bf16_t*)out, (const bf16_t*)in, pp, epochs, err, n,
                                            slot_bytes, rank, world);
  return (int)hipGetLastError();
}

}  // extern "C"
