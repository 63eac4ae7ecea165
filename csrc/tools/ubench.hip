// MFMA shape microbenchmark: v_mfma_f32_16x16x32_bf16 vs v_mfma_f32_32x32x16_bf16 on gfx950.
//
// Why it exists: every GEMM body in this repo (igemm, hconv, pgemm, pwconv, wgrad) issues the
// 16x16x32 form.  The two shapes take the same cycles per FLOP, but under load the chip holds
// a clock that depends on the instruction stream, so the choice is settled by wall time on
// random data, one wave per SIMD, the same output tile per wave (8 KB of fp32 accumulators):
//
//   SHAPE 16: 16 accumulators of 16x16 (4 fp32 per lane each)  -> 64 x 64 output per wave
//   SHAPE 32:  4 accumulators of 32x32 (16 fp32 per lane each) -> 64 x 64 output per wave
//
// Each loop trip is one 64-deep K step over the 64 x 64 tile (16x16x32: 2 k-halves x 16 MFMAs;
// 32x32x16: 4 k-quarters x 4 MFMAs) = 524,288 FLOP per wave per trip for both shapes.  LDS=1
// re-reads the A/B fragments from LDS every trip (ds_read_b128 at XOR-swizzled chunks; the
// LDS image holds random data), LDS=0 keeps them in registers.  bench/mfma_shape_bench.py times the launches.
//
// The accumulators are pinned to AGPRs after every k step (empty asm "+a"): unpinned, hipcc
// chose MFMA destinations that differ from their accumulator inputs and restored the loop-carried
// mapping with 112-120 v_accvgpr_read/write per trip of the 16x16x32 loop (none in the 32x32x16
// loop), which made the first version of this benchmark rank the 16x16x32 shape 1.3-1.65x slower
// for that reason alone.  With the pin, the LDS=1 loops of both shapes are MFMA + ds_read only;
// the LDS=0 16x16x32 loop still carries 56 v_accvgpr_read + 56 _write + 8 _mov per trip of
// 32 MFMAs (hipcc, loop-invariant operands; opaque operands or VGPR pins leave 24-120 of them),
// so its row (1,142 TF/s in profiles/r4/mfma_shape_bench.jsonl) measures the copies, not the
// instruction -- compare the LDS=1 rows, where both loops are MFMA + ds_read only.
#include "../common.h"

namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16;

template <int SHAPE, bool LDS>
__global__ __launch_bounds__(256, 1) void mfma_loop_kernel(const bf16* __restrict__ src, int trips,
                                                           float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) bf16 img[256 * 64];     // 32 KB of operands
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < 256 * 64 / 8; i += 256)
    *(bf16x8*)(img + i * 8) = *(const bf16x8*)(src + ((size_t)blockIdx.x * 2048 + i) * 8 % (1 << 20));
  __syncthreads();
  const int w = tid >> 6;
  const bf16* base = img + w * 64 * 64;   // this wave's 64 rows x 64 k
  if constexpr (SHAPE == 16) {
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 fa[2][4], fb[2][4];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = i * 16 + (lane & 15), ch = kk * 4 + (lane >> 4);
        fa[kk][i] = *(const bf16x8*)(base + row * 64 + ch * 8);
        fb[kk][i] = *(const bf16x8*)(base + ((row + 7) & 63) * 64 + ch * 8);
      }
    for (int t = 0; t < trips; ++t) {
      if constexpr (LDS) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = i * 16 + (lane & 15), ch = kk * 4 + (lane >> 4);
            fa[kk][i] = *(const bf16x8*)(base + row * 64 + (((ch + t) ^ row) & 7) * 8);
            fb[kk][i] = *(const bf16x8*)(base + ((row + 7) & 63) * 64 + (((ch + t) ^ (row + 7)) & 7) * 8);
          }
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kk][i], fb[kk][j], acc[i][j], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) asm volatile("" : "+a"(acc[i][j]));   // see header
      }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    out[blockIdx.x * 256 + tid] = s;
  } else {
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
    bf16x8 fa[4][2], fb[4][2];
#pragma unroll
    for (int kq = 0; kq < 4; ++kq)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        // 32x32x16: lane l holds row l & 31, k = 8 (l >> 5) .. + 7 of a 16-deep quarter
        const int row = i * 32 + (lane & 31), ch = kq * 2 + (lane >> 5);
        fa[kq][i] = *(const bf16x8*)(base + row * 64 + ch * 8);
        fb[kq][i] = *(const bf16x8*)(base + ((row + 7) & 63) * 64 + ch * 8);
      }
    for (int t = 0; t < trips; ++t) {
      if constexpr (LDS) {
#pragma unroll
        for (int kq = 0; kq < 4; ++kq)
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const int row = i * 32 + (lane & 31), ch = kq * 2 + (lane >> 5);
            fa[kq][i] = *(const bf16x8*)(base + row * 64 + (((ch + t) ^ row) & 7) * 8);
            fb[kq][i] = *(const bf16x8*)(base + ((row + 7) & 63) * 64 + (((ch + t) ^ (row + 7)) & 7) * 8);
          }
      }
#pragma unroll
      for (int kq = 0; kq < 4; ++kq)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[kq][i], fb[kq][j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) asm volatile("" : "+a"(acc[i][j]));
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) s += acc[i][j][q];
    out[blockIdx.x * 256 + tid] = s;
  }
}

}  // namespace

// shape 16 / 32, lds 0 / 1; src: >= 2 MB of bf16 (random), out: grid * 256 floats
// C ABI: this file is its own shared object (mercury_amd/_tools.so, loaded by ctypes from
// bench/mfma_shape_bench.py), not part of the production extension
extern "C" int ubench_mfma(int shape, int lds, const bf16* src, int trips, int grid, float* out,
                           hipStream_t st) {
#define UB_CASE(S_, L_)                                                                         \
  if (shape == S_ && lds == L_) {                                                               \
    hipLaunchKernelGGL((mfma_loop_kernel<S_, L_>), dim3(grid), dim3(256), 0, st, src, trips, out); \
    return 1;                                                                                   \
  }
  UB_CASE(16, false) UB_CASE(16, true) UB_CASE(32, false) UB_CASE(32, true)
#undef UB_CASE
  return 0;
}
