// Shared device helpers for the mercury_amd CDNA4 (gfx950) kernels.
//
// Conventions used by every kernel in csrc/:
//   * activations are NHWC bf16, channels padded to a multiple of 8 so every
//     (pixel, 8-channel chunk) is one 16-byte load;
//   * wave64 everywhere: lane = threadIdx.x & 63, cross-lane ops span 64 lanes;
//   * accumulation, BN statistics and optimizer state are fp32;
//   * all launchers take an explicit hipStream_t and never allocate or sync, so
//     every launch is capturable into a HIP graph.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define MA_DEV __device__ __forceinline__

// Timing probe only (bench/build_variant.py with -DMERCURY_SPREAD_PROBE=<floats>): forward BN
// statistics atomics go to one of 8 replicas by block (consumers read replica 0 only, so the
// statistics are WRONG) -- measures what the same-address atomic contention costs the step.
#ifdef MERCURY_SPREAD_PROBE
#define MA_SPREAD(p) ((p) + (size_t)(blockIdx.x & 7) * (MERCURY_SPREAD_PROBE))
#else
#define MA_SPREAD(p) (p)
#endif


MA_DEV float bf2f(bf16 x) { return (float)x; }
MA_DEV bf16 f2bf(float x) { return (bf16)x; }

MA_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
MA_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum over blockDim.x threads (multiple of 64). `red` is >= 16 floats of LDS.
MA_DEV float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

// ---------------------------------------------------------------------------------
// Philox4x32-10 counter-based RNG: stateless, so each (seed, stream, counter) gives
// an independent draw on any lane of any launch -- graph-replay safe.
// ---------------------------------------------------------------------------------
MA_DEV u32x4 philox4x32(u32x4 ctr, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * ctr.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * ctr.z;
    u32x4 n;
    n.x = (uint32_t)(p1 >> 32) ^ ctr.y ^ k0;
    n.y = (uint32_t)p1;
    n.z = (uint32_t)(p0 >> 32) ^ ctr.w ^ k1;
    n.w = (uint32_t)p0;
    ctr = n;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return ctr;
}
// x / d for 0 <= x < 2^24 and a wave-uniform divisor d via the float reciprocal (rcp is
// uniform, so it is computed once), with a one-step fix-up: ~6 VALU instead of the ~30 of an
// integer division.  Every pixel/row index of a conv GEMM is < 2^24.
MA_DEV int udiv24(int x, int d, float rcp) {
  int q = (int)((float)x * rcp);
  const int r = x - q * d;
  q += (r >= d) - (r < 0);
  return q;
}

MA_DEV float u01(uint32_t x) { return (x >> 8) * (1.0f / 16777216.0f); }  // [0,1)

// ---------------------------------------------------------------------------------
// Bijective hash permutation of [0, n): a 4-round Feistel network on the next power
// of two with cycle walking.  Gives every (seed, epoch) its own shuffle of a data
// shard without storing or sorting anything -- the device-side equivalent of a
// DataLoader(shuffle=True) epoch order.
// ---------------------------------------------------------------------------------
MA_DEV uint32_t feistel_round(uint32_t x, uint32_t key) {
  x ^= key;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
MA_DEV uint32_t permute_index(uint32_t i, uint32_t n, uint32_t seed, uint32_t epoch) {
  uint32_t bits = 2;
  while ((1u << bits) < n) ++bits;
  if (bits & 1) ++bits;
  const uint32_t half = bits >> 1, mask = (1u << half) - 1u;
  uint32_t x = i;
  do {
    uint32_t l = x >> half, r = x & mask;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t nl = r;
      r = l ^ (feistel_round(r, seed * 0x9E3779B9u + epoch * 0x85EBCA6Bu + k * 0xC2B2AE35u) & mask);
      l = nl;
    }
    x = (l << half) | r;
  } while (x >= n);
  return x;
}

#define HIP_LAUNCH_CHECK() (void)0
