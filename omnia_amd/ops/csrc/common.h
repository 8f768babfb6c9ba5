// Shared device helpers for the omnia_amd CDNA4 (gfx950) kernels.
//
// Everything here is written for 64-lane wavefronts and the gfx950 MFMA /
// LDS model (see docs/KERNELS.md).  No CUDA spellings, no dual paths.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace omnia {

using bf16_t = uint16_t;  // raw bf16 storage
typedef short short8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float float4v __attribute__((ext_vector_type(4)));
typedef float float16v __attribute__((ext_vector_type(16)));
typedef unsigned int uint4v __attribute__((ext_vector_type(4)));
typedef unsigned int uint2v __attribute__((ext_vector_type(2)));

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(uint16_t x) {
  return __uint_as_float(((uint32_t)x) << 16);
}

// round-to-nearest-even f32 -> bf16 (inputs are finite on every hot path)
__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// two f32 -> packed bf16x2 (low = a)
__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block-wide sum; `scratch` holds >= blockDim/64 floats
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += scratch[i];
  return t;
}

__device__ __forceinline__ float block_max(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float t = -INFINITY;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, scratch[i]);
  return t;
}

// 64-bit mix (splitmix64 finaliser) -> counter-based RNG for the sampler
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t ctr) {
  uint64_t r = mix64(seed ^ mix64(ctr));
  // 24 random mantissa bits, strictly inside (0,1)
  return ((float)(r >> 40) + 0.5f) * (1.0f / 16777216.0f);
}

// XCD-aware bijective remap of a 1-D block id: blocks b and b+8 share an XCD
// under round-robin dispatch; give each XCD a contiguous chunk of the logical
// grid so neighbouring tiles share its L2 (guide T1, bijective form).
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

}  // namespace omnia
