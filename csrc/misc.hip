// Remaining layer kernels: pooling (VGG / ImageNet stem), stochastic quantisation (`util.py:65-70`) and
// NCHW fp32 -> NHWC bf16 layout conversion for host-fed tensors.
#include <stdexcept>

#include "common.h"
#include "kernels.h"

namespace {
constexpr int NT = 256;

// --------------------------------------------------------------- pooling
// One thread per (output pixel, 8-channel chunk): 16-byte loads and stores, 32-bit index math
// (a 64-bit div/mod is a ~100-instruction call; the ImageNet-stem pool at B=1280 was VALU-bound
// on it).  The max pool records the window tap r*k+s of each maximum as one byte per channel
// (first maximum in scan order, like torch), so the backward reads 8 taps as one 8-byte word.
MA_DEV void ld8(const float* p, float (&v)[8]) {     // 8 floats as two 16-byte loads
  const float4 x = *(const float4*)p, y = *(const float4*)(p + 4);
  v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
}
MA_DEV float pool_act(float v, int act) {
  if (act == 1) return fmaxf(v, 0.f);
  if (act == 2) return fminf(fmaxf(v, 0.f), 6.f);
  return v;
}

// KS > 0: the window size is a compile-time constant and all KS*KS tap loads are issued
// before the first is used (out-of-image taps load a clamped in-image pixel and are masked);
// KS == 0: runtime window, one tap at a time.  MODE: 0 max, 1 max + argmax, 2 max of
// act(BN(x)), 3 average.  MODE 2 keeps the max AND the min of the raw values and transforms
// once: act(sc*x + sh) and its bf16 rounding are monotone in x -- non-decreasing for sc >= 0
// (take the max), non-increasing for sc < 0 (take the min) -- so the result equals the max of
// bn_apply's bf16 outputs, at a ninth of the transform work (the kernel was VALU-bound).
template <int KS, int MODE>
__global__ __launch_bounds__(NT) void pool2d_fwd_kernel(PoolArgs a) {
  const unsigned C8 = (unsigned)a.C >> 3;
  const unsigned total = (unsigned)a.N * a.P * a.Q * C8;
  const unsigned i = blockIdx.x * NT + threadIdx.x;
  if (i >= total) return;
  const unsigned c8 = i % C8;
  unsigned pix = i / C8;
  const int q = (int)(pix % (unsigned)a.Q);
  pix /= (unsigned)a.Q;
  const int p = (int)(pix % (unsigned)a.P), n = (int)(pix / (unsigned)a.P);
  const int c = (int)c8 * 8;
  const int k = KS > 0 ? KS : a.k;
  const int h0 = p * a.stride - a.pad, w0 = q * a.stride - a.pad;
  const bf16* xn = a.x + (size_t)n * a.H * a.W * a.C + c;
  constexpr int NV = KS > 0 ? KS * KS : 1;
  bf16x8 v[NV];
  if (KS > 0) {
#pragma unroll
    for (int t = 0; t < NV; ++t) {
      const int h = min(max(h0 + t / (KS > 0 ? KS : 1), 0), a.H - 1);
      const int w = min(max(w0 + t % (KS > 0 ? KS : 1), 0), a.W - 1);
      v[t] = *(const bf16x8*)(xn + (unsigned)(h * a.W + w) * (unsigned)a.C);
    }
  }
  float acc[8], mn[8];
  int arg[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    acc[j] = MODE == 3 ? 0.f : -3.4e38f;
    mn[j] = 3.4e38f;
    arg[j] = 0;
  }
#pragma unroll
  for (int t = 0; t < (KS > 0 ? NV : 1); ++t) {
    for (int tt = (KS > 0 ? t : 0); tt < (KS > 0 ? t + 1 : k * k); ++tt) {
      const int h = h0 + tt / k, w = w0 + tt % k;
      if (h < 0 || h >= a.H || w < 0 || w >= a.W) continue;
      const bf16x8 x = KS > 0 ? v[t] : *(const bf16x8*)(xn + (unsigned)(h * a.W + w) * (unsigned)a.C);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float f = bf2f(x[j]);
        if (MODE == 3) {
          acc[j] += f;
        } else if (MODE == 1) {
          if (f > acc[j]) {
            acc[j] = f;
            arg[j] = tt;
          }
        } else {
          acc[j] = fmaxf(acc[j], f);
          if (MODE == 2) mn[j] = fminf(mn[j], f);
        }
      }
    }
  }
  if (MODE == 2) {
    // BN of the input: per-channel scale/shift of this image's ghost group
    const bool run = a.stats == nullptr;
    const int g = a.group_imgs > 0 ? n / a.group_imgs : 0;
    const float inv = 1.f / (float)((a.group_imgs > 0 ? a.group_imgs : a.N) * a.H * a.W);
    const float* s0 = run ? a.rmean + c : a.stats + (size_t)g * 2 * a.C + c;
    const float* s1 = run ? a.rvar + c : s0 + a.C;
    float m8[8], v8[8], g8[8], b8[8];
    ld8(s0, m8);
    ld8(s1, v8);
    ld8(a.gamma + c, g8);
    ld8(a.beta + c, b8);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float mean = m8[j], var = v8[j];
      if (!run) {
        mean *= inv;
        var = fmaxf(var * inv - mean * mean, 0.f);
      }
      const float sc = g8[j] * rsqrtf(var + a.eps);
      const float sh = b8[j] - mean * sc;
      acc[j] = pool_act((sc >= 0.f ? acc[j] : mn[j]) * sc + sh, a.act);
    }
  }
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = f2bf(MODE == 3 ? acc[j] / (float)(k * k) : acc[j]);
  *(bf16x8*)(a.y + (size_t)i * 8) = o;
  if (MODE == 1) {
    uint2 t;
    t.x = (uint32_t)arg[0] | ((uint32_t)arg[1] << 8) | ((uint32_t)arg[2] << 16) |
          ((uint32_t)arg[3] << 24);
    t.y = (uint32_t)arg[4] | ((uint32_t)arg[5] << 8) | ((uint32_t)arg[6] << 16) |
          ((uint32_t)arg[7] << 24);
    *(uint2*)(a.argmax + (size_t)i * 8) = t;
  }
}

template <int MODE>
void pool2d_fwd_mode(const PoolArgs& a, dim3 grid, hipStream_t st) {
  if (a.k == 3)
    hipLaunchKernelGGL((pool2d_fwd_kernel<3, MODE>), grid, dim3(NT), 0, st, a);
  else if (a.k == 2)
    hipLaunchKernelGGL((pool2d_fwd_kernel<2, MODE>), grid, dim3(NT), 0, st, a);
  else
    hipLaunchKernelGGL((pool2d_fwd_kernel<0, MODE>), grid, dim3(NT), 0, st, a);
}

// gather form, one thread per (input pixel, 8 channels): every input element sums the output
// gradients of the windows whose recorded maximum is this element's tap
__global__ __launch_bounds__(NT) void maxpool_bwd_kernel(PoolArgs a, const bf16* dy, bf16* dx) {
  const unsigned C8 = (unsigned)a.C >> 3;
  const unsigned total = (unsigned)a.N * a.H * a.W * C8;
  const unsigned i = blockIdx.x * NT + threadIdx.x;
  if (i >= total) return;
  const unsigned c8 = i % C8;
  unsigned pix = i / C8;
  const int w = (int)(pix % (unsigned)a.W);
  pix /= (unsigned)a.W;
  const int h = (int)(pix % (unsigned)a.H), n = (int)(pix / (unsigned)a.H);
  float s[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s[k] = 0.f;
  const int p0 = max(0, (h + a.pad - a.k + a.stride) / a.stride), p1 = min(a.P - 1, (h + a.pad) / a.stride);
  const int q0 = max(0, (w + a.pad - a.k + a.stride) / a.stride), q1 = min(a.Q - 1, (w + a.pad) / a.stride);
  for (int p = p0; p <= p1; ++p)
    for (int q = q0; q <= q1; ++q) {
      const size_t o = ((size_t)(n * a.P + p) * a.Q + q) * a.C + c8 * 8;
      const uint32_t tap = (uint32_t)((h - (p * a.stride - a.pad)) * a.k + (w - (q * a.stride - a.pad)));
      const uint2 t = *(const uint2*)(a.argmax + o);
      const bf16x8 g = *(const bf16x8*)(dy + o);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t b = ((k < 4 ? t.x : t.y) >> (8 * (k & 3))) & 255u;
        if (b == tap) s[k] += bf2f(g[k]);
      }
    }
  bf16x8 o;
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] = f2bf(s[k]);
  *(bf16x8*)(dx + (size_t)i * 8) = o;
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

// Ternary gradient wire (the quantiser above as a compressed all-reduce): element i of a
// bucket travels as 2 bits c in {0: 0, 1: +1, 2: -1} drawn with P(|c| = 1) = |x| / max|x|, and
// the bucket's max|x| as one fp32 word -- 16 elements per int32 word, message = 1 + n/16 words.
// Unbiased per rank (E[scale * c] = x); the receiver sums scale_r * c_r over the W messages.
__global__ __launch_bounds__(NT) void tern_pack_kernel(const float* x, long long n,
                                                       const float* amax, uint32_t seed,
                                                       uint64_t counter, const long long* dctr,
                                                       uint32_t* words) {
  const long long j = (long long)blockIdx.x * NT + threadIdx.x;   // word index
  // graph-replayed steps: the Philox stream comes from the device step counter (a captured
  // host counter would replay the same stream every step): the step in the low word, the bucket
  // index in the high word -- no two (step, bucket) pairs share a stream for < 2^32 buckets
  if (dctr) counter = ((uint64_t)(uint32_t)counter << 32) | (uint64_t)(uint32_t)dctr[0];
  const long long nw = (n + 15) / 16;
  const float m = *amax;
  if (j == 0) words[0] = __float_as_uint(m);
  if (j >= nw) return;
  uint32_t w = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const long long e0 = j * 16 + q * 4;
    const u32x4 r = philox4x32(u32x4{(uint32_t)e0, (uint32_t)(e0 >> 32), (uint32_t)counter,
                                     (uint32_t)(counter >> 32)}, seed, 0x85EBCA6Bu);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const long long e = e0 + k;
      if (e < n) {
        const float v = x[e];
        const uint32_t rk = k == 0 ? r.x : (k == 1 ? r.y : (k == 2 ? r.z : r.w));
        const bool keep = m > 0.f && u01(rk) < fabsf(v) / m;
        const uint32_t c = keep ? (v > 0.f ? 1u : (v < 0.f ? 2u : 0u)) : 0u;
        w |= c << (2 * (q * 4 + k));
      }
    }
  }
  words[1 + j] = w;
}

// out[i] = scale * sum_r max_r * c_r[i] over W gathered messages of nw words each
__global__ __launch_bounds__(NT) void tern_unpack_kernel(const uint32_t* msgs, int W, long long nw,
                                                         long long n, float scale, float* out) {
  const long long j = (long long)blockIdx.x * NT + threadIdx.x;
  if (j >= nw - 1) return;
  float acc[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) acc[k] = 0.f;
  for (int r = 0; r < W; ++r) {
    const uint32_t* m = msgs + (size_t)r * nw;
    const float mx = __uint_as_float(m[0]);
    const uint32_t w = m[1 + j];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t c = (w >> (2 * k)) & 3u;
      acc[k] += c == 1u ? mx : (c == 2u ? -mx : 0.f);
    }
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const long long e = j * 16 + k;
    if (e < n) out[e] = acc[k] * scale;
  }
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
  if (a.C % 8 || (long long)a.N * a.H * a.W * a.C >= (1ll << 32) || total >= (1ll << 31)) {
    throw std::runtime_error("pool2d_fwd: C % 8 or the 32-bit index range violated");
  }
  const dim3 grid((unsigned)((total + NT - 1) / NT));
  const bool bn = a.stats != nullptr || a.rmean != nullptr;
  if (!a.is_max && (bn || a.argmax))
    throw std::runtime_error("pool2d_fwd: BN / argmax only with the max pool");
  if (bn && a.argmax)
    throw std::runtime_error("pool2d_fwd: the BN-applying pool records no argmax");
  if (!a.is_max)
    pool2d_fwd_mode<3>(a, grid, st);
  else if (bn)
    pool2d_fwd_mode<2>(a, grid, st);
  else if (a.argmax)
    pool2d_fwd_mode<1>(a, grid, st);
  else
    pool2d_fwd_mode<0>(a, grid, st);
}
void maxpool2d_bwd_launch(const PoolArgs& a, const bf16* dy, bf16* dx, hipStream_t st) {
  const long long total = (long long)a.N * a.H * a.W * (a.C / 8);
  if (a.C % 8 || total >= (1ll << 31) || a.k * a.k > 255) {
    throw std::runtime_error("maxpool2d_bwd: C % 8, the 32-bit index range or window size violated");
  }
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
void tern_pack_launch(const float* x, long long n, float* absmax_ws, uint32_t seed,
                      uint64_t counter, const long long* dctr, uint32_t* words, hipStream_t st) {
  hipMemsetAsync(absmax_ws, 0, sizeof(float), st);
  const long long blocks = (n + NT - 1) / NT;
  hipLaunchKernelGGL(absmax_kernel, dim3((unsigned)(blocks > 1024 ? 1024 : blocks)), dim3(NT), 0, st,
                     x, n, absmax_ws);
  const long long nw = (n + 15) / 16;
  hipLaunchKernelGGL(tern_pack_kernel, dim3((unsigned)((nw + NT - 1) / NT)), dim3(NT), 0, st, x, n,
                     absmax_ws, seed, counter, dctr, words);
}
void tern_unpack_launch(const uint32_t* msgs, int W, long long n, float scale, float* out,
                        hipStream_t st) {
  const long long nw = 1 + (n + 15) / 16;
  hipLaunchKernelGGL(tern_unpack_kernel, dim3((unsigned)((nw - 1 + NT - 1) / NT)), dim3(NT), 0, st,
                     msgs, W, nw, n, scale, out);
}
void nchw_to_nhwc8_launch(const float* x, bf16* y, int N, int C, int H, int W, int Cpad,
                          hipStream_t st) {
  const long long total = (long long)N * H * W * Cpad;
  hipLaunchKernelGGL(nchw_to_nhwc8_kernel, dim3((unsigned)((total + NT - 1) / NT)), dim3(NT), 0, st, x,
                     y, N, C, H, W, Cpad);
}
