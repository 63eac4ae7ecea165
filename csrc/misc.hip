// Remaining layer kernels: pooling (VGG / ImageNet stem), stochastic quantisation (`util.py:65-70`) and
// NCHW fp32 -> NHWC bf16 layout conversion for host-fed tensors.
#include "common.h"
#include "kernels.h"

namespace {
constexpr int NT = 256;

// --------------------------------------------------------------- pooling
__global__ __launch_bounds__(NT) void pool2d_fwd_kernel(PoolArgs a) {
  const int C8 = a.C >> 3;
  const long long total = (long long)a.N * a.P * a.Q * C8;
  const long long i = (long long)blockIdx.x * NT + threadIdx.x;
  if (i >= total) return;
  const int c8 = (int)(i % C8);
  const long long pix = i / C8;
  const int q = (int)(pix % a.Q), p = (int)((pix / a.Q) % a.P), n = (int)(pix / ((long long)a.P * a.Q));
  float acc[8];
  int arg[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    acc[k] = a.is_max ? -3.4e38f : 0.f;
    arg[k] = -1;
  }
  int cnt = 0;
  for (int r = 0; r < a.k; ++r) {
    const int h = p * a.stride - a.pad + r;
    if (h < 0 || h >= a.H) continue;
    for (int s = 0; s < a.k; ++s) {
      const int w = q * a.stride - a.pad + s;
      if (w < 0 || w >= a.W) continue;
      const size_t base = ((size_t)(n * a.H + h) * a.W + w) * a.C + c8 * 8;
      const bf16x8 v = *(const bf16x8*)(a.x + base);
      ++cnt;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float f = bf2f(v[k]);
        if (a.is_max) {
          if (f > acc[k]) {
            acc[k] = f;
            arg[k] = (int)(base + k);
          }
        } else {
          acc[k] += f;
        }
      }
    }
  }
  bf16x8 o;
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] = f2bf(a.is_max ? acc[k] : acc[k] / (float)(a.k * a.k));
  *(bf16x8*)(a.y + i * 8) = o;
  if (a.argmax) {
#pragma unroll
    for (int k = 0; k < 8; ++k) a.argmax[i * 8 + k] = arg[k];
  }
}

// gather form: every input element sums the output gradients whose argmax it is
__global__ __launch_bounds__(NT) void maxpool_bwd_kernel(PoolArgs a, const bf16* dy, bf16* dx) {
  const long long total = (long long)a.N * a.H * a.W * a.C;
  const long long i = (long long)blockIdx.x * NT + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % a.C);
  const long long pix = i / a.C;
  const int w = (int)(pix % a.W), h = (int)((pix / a.W) % a.H), n = (int)(pix / ((long long)a.H * a.W));
  float s = 0.f;
  const int p0 = max(0, (h + a.pad - a.k + a.stride) / a.stride), p1 = min(a.P - 1, (h + a.pad) / a.stride);
  const int q0 = max(0, (w + a.pad - a.k + a.stride) / a.stride), q1 = min(a.Q - 1, (w + a.pad) / a.stride);
  for (int p = p0; p <= p1; ++p)
    for (int q = q0; q <= q1; ++q) {
      const size_t o = ((size_t)(n * a.P + p) * a.Q + q) * a.C + c;
      if (a.argmax[o] == (int)i) s += bf2f(dy[o]);
    }
  dx[i] = f2bf(s);
}

// --------------------------------------------------------------- quantisation
__global__ __launch_bounds__(NT) void absmax_kernel(const float* x, long long n, float* out) {
  float m = 0.f;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT)
    m = fmaxf(m, fabsf(x[i]));
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) atomicMax((unsigned int*)out, __float_as_uint(m));
}
__global__ __launch_bounds__(NT) void quantize_kernel(const float* x, float* y, const float* amax,
                                                      long long n, uint32_t seed, uint64_t counter) {
  const long long i = (long long)blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  const float m = *amax;
  const u32x4 r = philox4x32(u32x4{(uint32_t)i, (uint32_t)(i >> 32), (uint32_t)counter,
                                   (uint32_t)(counter >> 32)}, seed, 0x9E3779B9u);
  const float v = x[i];
  const float keep = (m > 0.f && u01(r.x) < fabsf(v) / m) ? 1.f : 0.f;
  y[i] = (v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f)) * m * keep;
}

__global__ __launch_bounds__(NT) void nchw_to_nhwc8_kernel(const float* x, bf16* y, int N, int C, int H,
                                                           int W, int Cpad) {
  const long long total = (long long)N * H * W * Cpad;
  const long long i = (long long)blockIdx.x * NT + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % Cpad);
  const long long pix = i / Cpad;
  const int w = (int)(pix % W), h = (int)((pix / W) % H), n = (int)(pix / ((long long)H * W));
  y[i] = c < C ? f2bf(x[(((size_t)n * C + c) * H + h) * W + w]) : f2bf(0.f);
}
}  // namespace

void pool2d_fwd_launch(const PoolArgs& a, hipStream_t st) {
  const long long total = (long long)a.N * a.P * a.Q * (a.C / 8);
  hipLaunchKernelGGL(pool2d_fwd_kernel, dim3((unsigned)((total + NT - 1) / NT)), dim3(NT), 0, st, a);
}
void maxpool2d_bwd_launch(const PoolArgs& a, const bf16* dy, bf16* dx, hipStream_t st) {
  const long long total = (long long)a.N * a.H * a.W * a.C;
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3((unsigned)((total + NT - 1) / NT)), dim3(NT), 0, st, a,
                     dy, dx);
}
void quantize_launch(const float* x, float* out, float* absmax_ws, long long n, uint32_t seed,
                     uint64_t counter, hipStream_t st) {
  hipMemsetAsync(absmax_ws, 0, sizeof(float), st);
  long long blocks = (n + NT - 1) / NT;
  hipLaunchKernelGGL(absmax_kernel, dim3((unsigned)(blocks > 1024 ? 1024 : blocks)), dim3(NT), 0, st, x,
                     n, absmax_ws);
  hipLaunchKernelGGL(quantize_kernel, dim3((unsigned)blocks), dim3(NT), 0, st, x, out, absmax_ws, n,
                     seed, counter);
}
void nchw_to_nhwc8_launch(const float* x, bf16* y, int N, int C, int H, int W, int Cpad,
                          hipStream_t st) {
  const long long total = (long long)N * H * W * Cpad;
  hipLaunchKernelGGL(nchw_to_nhwc8_kernel, dim3((unsigned)((total + NT - 1) / NT)), dim3(NT), 0, st, x,
                     y, N, C, H, W, Cpad);
}
