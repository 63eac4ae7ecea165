// Remaining layer kernels: pooling (VGG / ImageNet stem), depthwise 3x3 conv
// (MobileNetV2), stochastic quantisation (`util.py:65-70`) and
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

// --------------------------------------------------------------- depthwise 3x3
// One block per (image, channel-block of 8*32 channels); threads = 8 pixel lanes x 32 chunks.
__global__ __launch_bounds__(NT) void dw_fwd_kernel(DwArgs a) {
  __shared__ float red[2 * 1024];
  const int C8 = a.C >> 3;
  const int n = blockIdx.x;
  for (int i = threadIdx.x; i < 2 * a.C; i += NT) red[i] = 0.f;
  __syncthreads();
  const int items = a.P * a.Q * C8;
  float s[8], ss[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s[k] = ss[k] = 0.f;
  int c8_last = -1;
  for (int it = threadIdx.x; it < items; it += NT) {
    const int c8 = it % C8, pq = it / C8;
    if (c8 != c8_last && c8_last >= 0 && a.stats) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        atomicAdd(&red[c8_last * 8 + k], s[k]);
        atomicAdd(&red[a.C + c8_last * 8 + k], ss[k]);
        s[k] = ss[k] = 0.f;
      }
    }
    c8_last = c8;
    const int p = pq / a.Q, q = pq - p * a.Q;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int r = 0; r < 3; ++r) {
      const int h = p * a.stride - a.pad + r;
      if (h < 0 || h >= a.H) continue;
      for (int t = 0; t < 3; ++t) {
        const int w = q * a.stride - a.pad + t;
        if (w < 0 || w >= a.W) continue;
        const bf16x8 v = *(const bf16x8*)(a.x + ((size_t)(n * a.H + h) * a.W + w) * a.C + c8 * 8);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += bf2f(v[k]) * a.w[(c8 * 8 + k) * 9 + r * 3 + t];
      }
    }
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      o[k] = f2bf(acc[k]);
      const float f = bf2f(o[k]);
      s[k] += f;
      ss[k] += f * f;
    }
    *(bf16x8*)(a.y + ((size_t)(n * a.P + p) * a.Q + q) * a.C + c8 * 8) = o;
  }
  if (a.stats) {
    if (c8_last >= 0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        atomicAdd(&red[c8_last * 8 + k], s[k]);
        atomicAdd(&red[a.C + c8_last * 8 + k], ss[k]);
      }
    }
    __syncthreads();
    const int g = (n * a.P * a.Q) / a.group_rows;
    float* dst = a.stats + (size_t)g * 2 * a.C;
    for (int c = threadIdx.x; c < a.C; c += NT) {
      atomicAdd(dst + c, red[c]);
      atomicAdd(dst + a.C + c, red[a.C + c]);
    }
  }
}

__global__ __launch_bounds__(NT) void dw_dgrad_kernel(const bf16* dy, const float* w, bf16* dx, int N,
                                                      int H, int W, int C, int P, int Q, int stride,
                                                      int pad) {
  const int C8 = C >> 3;
  const long long total = (long long)N * H * W * C8;
  const long long i = (long long)blockIdx.x * NT + threadIdx.x;
  if (i >= total) return;
  const int c8 = (int)(i % C8);
  const long long pix = i / C8;
  const int x = (int)(pix % W), y = (int)((pix / W) % H), n = (int)(pix / ((long long)H * W));
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int r = 0; r < 3; ++r) {
    const int hp = y + pad - r;
    if (hp < 0 || hp % stride) continue;
    const int p = hp / stride;
    if (p >= P) continue;
    for (int t = 0; t < 3; ++t) {
      const int wp = x + pad - t;
      if (wp < 0 || wp % stride) continue;
      const int q = wp / stride;
      if (q >= Q) continue;
      const bf16x8 v = *(const bf16x8*)(dy + ((size_t)(n * P + p) * Q + q) * C + c8 * 8);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += bf2f(v[k]) * w[(c8 * 8 + k) * 9 + r * 3 + t];
    }
  }
  bf16x8 o;
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] = f2bf(acc[k]);
  *(bf16x8*)(dx + i * 8) = o;
}

// one block per image; each thread accumulates 9 taps x 8 channels for its chunk
__global__ __launch_bounds__(NT) void dw_wgrad_kernel(const bf16* dy, const bf16* x, float* dw, int N,
                                                      int H, int W, int C, int P, int Q, int stride,
                                                      int pad) {
  const int C8 = C >> 3;
  const int n = blockIdx.x;
  const int lanes = NT / C8 > 0 ? NT / C8 : 1;
  const int sub = threadIdx.x / C8;
  if (sub >= lanes) return;
  for (int c8 = threadIdx.x % C8; c8 < C8; c8 += NT) {
    float acc[9][8];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[t][k] = 0.f;
    for (int pq = sub; pq < P * Q; pq += lanes) {
      const int p = pq / Q, q = pq - p * Q;
      const bf16x8 g = *(const bf16x8*)(dy + ((size_t)(n * P + p) * Q + q) * C + c8 * 8);
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int h = p * stride - pad + r;
        if (h < 0 || h >= H) continue;
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          const int w = q * stride - pad + t;
          if (w < 0 || w >= W) continue;
          const bf16x8 v = *(const bf16x8*)(x + ((size_t)(n * H + h) * W + w) * C + c8 * 8);
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[r * 3 + t][k] += bf2f(g[k]) * bf2f(v[k]);
        }
      }
    }
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int k = 0; k < 8; ++k) atomicAdd(&dw[(c8 * 8 + k) * 9 + t], acc[t][k]);
  }
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
void dwconv_fwd_launch(const DwArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(dw_fwd_kernel, dim3(a.N), dim3(NT), 0, st, a);
}
void dwconv_dgrad_launch(const bf16* dy, const float* w, bf16* dx, int N, int H, int W, int C, int P,
                         int Q, int stride, int pad, hipStream_t st) {
  const long long total = (long long)N * H * W * (C / 8);
  hipLaunchKernelGGL(dw_dgrad_kernel, dim3((unsigned)((total + NT - 1) / NT)), dim3(NT), 0, st, dy, w,
                     dx, N, H, W, C, P, Q, stride, pad);
}
void dwconv_wgrad_launch(const bf16* dy, const bf16* x, float* dw, int N, int H, int W, int C, int P,
                         int Q, int stride, int pad, hipStream_t st) {
  hipLaunchKernelGGL(dw_wgrad_kernel, dim3(N), dim3(NT), 0, st, dy, x, dw, N, H, W, C, P, Q, stride,
                     pad);
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
