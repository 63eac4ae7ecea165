// Stem convolution: 1-4 input channels (RGB images, single-channel spectrograms), the first layer
// of every model family (`pytorch_model.py:72` CIFAR 3x3 3 -> 64, `:89` ImageNet 7x7/2 3 -> 64,
// MobileNetV2's 3x3 3 -> 32, the speech VGG's 3x3 1 -> 64).
//
// A generic implicit GEMM pads the 3 channels to 8 per tap, so half of every MFMA k-slice
// multiplies zeros and a 7x7 tap window is 13 k-steps deep.  Here the reduction packs
// (tap, channel) pairs densely -- k = tap * 4 + c, channel 3 a zero lane -- so a 7x7 window is
// 196 -> 224 k (7 steps of 32) and a 3x3 window 36 -> 64 (2 steps).
//
// A block owns one image and walks TPB output tiles of 16 x 16 pixels:
//   * the weights [K][taps][4] are staged ONCE per block into LDS (64-byte swizzled rows);
//   * each tile's input window ((16-1)*stride + R)^2 pixels x 4 channels is staged in LDS, zero
//     outside the image, and the MFMA B fragments (8 k = 2 taps x 4 channels of one pixel) are
//     two 8-byte LDS reads at per-lane tap offsets computed once;
//   * MFMA 16x16x32 with the weights as A: each lane ends up with 4 consecutive output channels
//     of one pixel, stored as one 8-byte NHWC write (+ bias), and its BN sums run in registers
//     across the block's tiles: one DPP row reduction, one LDS pass and one atomic pair per
//     channel per block (a block never leaves its image, so never its ghost-BN group).
#include "common.h"
#include "kernels.h"

namespace {

constexpr int ST_T = 16;         // output tile edge (pixels)
constexpr int ST_NT = 256;       // 4 waves: wave w computes tile rows 4w .. 4w + 3

MA_DEV float st_row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  return v;
}
typedef uint32_t st_u32x2 __attribute__((ext_vector_type(2)));

// Output-channel order of the weight rows in LDS: within every 32 rows, row h * 16 + 4 q + j
// (fragment half h, lane group q, accumulator element j) holds channel 8 q + 4 h + j, so a lane's
// accumulators of fragments (2t, 2t + 1) are 8 consecutive channels of its pixel and leave as
// one 16-byte store (16 pixels x 64 bytes per wave instruction instead of x 32: the ResNet-50
// stem writes 2 GB at B = 1280)
MA_DEV int st_perm(int r) {
  const int r5 = r & 31;
  return (r & ~31) | (((r5 >> 2) & 3) << 3) | ((r5 >> 4) << 2) | (r5 & 3);
}

// R x R taps, stride S, K = 16 * KT output channels
template <int R, int S, int KT>
__global__ __launch_bounds__(ST_NT) void stem_kernel(StemArgs a) {
  static_assert(KT % 2 == 0, "fragment pairs (st_perm)");
  constexpr int RR = R * R;
  constexpr int KS = (RR * 4 + 31) / 32;           // 32-deep k-steps
  constexpr int K = 16 * KT;
  constexpr int PW = (ST_T - 1) * S + R;           // input window edge
  constexpr int WB = KS * K * 64;                  // weight bytes in LDS
  __shared__ __attribute__((aligned(16))) char sw[WB];
  __shared__ __attribute__((aligned(16))) st_u32x2 sp[PW * PW];
  __shared__ float red[4][2][K];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int tq = (a.Q + ST_T - 1) / ST_T, tpi = tq * ((a.P + ST_T - 1) / ST_T);
  const int n = blockIdx.x / a.blocks_per_img;
  const int t0 = (blockIdx.x - n * a.blocks_per_img) * a.tpb;
  const int t1 = min(t0 + a.tpb, tpi);

  // weights [K][RR][8] (channels 0..3 used) -> LDS [ks][k][32], chunk c of row k at c ^ ((k>>1)&3)
  for (int i = tid; i < K * KS * 8; i += ST_NT) {
    const int k = i / (KS * 8), t = i - k * (KS * 8);
    st_u32x2 v = {0u, 0u};
    if (t < RR) v = *(const st_u32x2*)(a.w + ((size_t)st_perm(k) * RR + t) * 8);
    const int ks = t >> 3, ch = (t & 7) >> 1;
    *(st_u32x2*)(sw + (ks * K + k) * 64 + ((ch ^ ((k >> 1) & 3)) * 16) + (t & 1) * 8) = v;
  }
  // per-lane LDS offsets of the two taps of each k-step (pixel-relative, in 8-byte units); -1
  // marks a k-padding tap past R * R (contributes zeros)
  int toff[KS][2];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int t = ks * 8 + (lane >> 4) * 2 + h;
      toff[ks][h] = t < RR ? (t / R) * PW + (t % R) : -1;
    }
  // weight fragment offsets: out-channel row 16 * kt + (lane & 15), logical chunk lane >> 4
  const int wfo = (lane & 15) * 64 + 16 * ((lane >> 4) ^ ((lane >> 1) & 3));

  float s[KT][4], ss[KT][4];
#pragma unroll
  for (int kt = 0; kt < KT; ++kt)
#pragma unroll
    for (int j = 0; j < 4; ++j) s[kt][j] = ss[kt][j] = 0.f;
  f32x4 bias[KT];
#pragma unroll
  for (int kt = 0; kt < KT; ++kt)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      bias[kt][j] = a.bias ? a.bias[st_perm(16 * kt + 4 * (lane >> 4) + j)] : 0.f;

  const st_u32x2* xin = (const st_u32x2*)a.x + (size_t)n * a.H * a.W * 2;   // 16-byte pixels
  // the next tile's input window is loaded into registers while this tile computes
  constexpr int NPT = (PW * PW + ST_NT - 1) / ST_NT;
  st_u32x2 pv[NPT];
  auto load_window = [&](int t) {
    const int p0 = (t / tq) * ST_T, q0 = (t % tq) * ST_T;
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
      const int i = tid + j * ST_NT;
      const int r = i / PW, c = i - r * PW;
      const int ih = p0 * S - a.pad + r, iw = q0 * S - a.pad + c;
      const bool ok = i < PW * PW && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
      pv[j] = ok ? xin[((size_t)ih * a.W + iw) * 2] : st_u32x2{0u, 0u};
    }
  };
  if (t0 < t1) load_window(t0);
  for (int t = t0; t < t1; ++t) {
    const int p0 = (t / tq) * ST_T, q0 = (t % tq) * ST_T;
    __syncthreads();                                 // previous tile's window reads done
#pragma unroll
    for (int j = 0; j < NPT; ++j)
      if (tid + j * ST_NT < PW * PW) sp[tid + j * ST_NT] = pv[j];
    __syncthreads();
    if (t + 1 < t1) load_window(t + 1);
    f32x4 acc[4][KT];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) acc[g][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 fw[KT];
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) fw[kt] = *(const bf16x8*)(sw + (ks * K + 16 * kt) * 64 + wfo);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        // pixel (tile row 4w + g, column lane & 15): window origin (row * S, col * S)
        const int base = ((4 * w + g) * S) * PW + (lane & 15) * S;
        st_u32x2 lo = {0u, 0u}, hi = {0u, 0u};
        if (toff[ks][0] >= 0) lo = sp[base + toff[ks][0]];
        if (toff[ks][1] >= 0) hi = sp[base + toff[ks][1]];
        const bf16x8 fx = __builtin_bit_cast(bf16x8, u32x4{lo[0], lo[1], hi[0], hi[1]});
#pragma unroll
        for (int kt = 0; kt < KT; ++kt)
          acc[g][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[kt], fx, acc[g][kt], 0, 0, 0);
      }
    }
    // epilogue: (+ bias) -> bf16 NHWC (one 16-byte store per fragment pair, st_perm), BN sums
    // of the rounded values
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int p = p0 + 4 * w + g, q = q0 + (lane & 15);
      const bool ok = p < a.P && q < a.Q;
      bf16* yp = a.y + (((size_t)n * a.P + p) * a.Q + q) * K + 8 * (lane >> 4);
#pragma unroll
      for (int tp = 0; tp < KT / 2; ++tp) {
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          o[j] = f2bf(acc[g][2 * tp][j] + bias[2 * tp][j]);
          o[4 + j] = f2bf(acc[g][2 * tp + 1][j] + bias[2 * tp + 1][j]);
        }
        if (ok) {
          *(bf16x8*)(yp + 32 * tp) = o;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float f = bf2f(o[j]), f2 = bf2f(o[4 + j]);
            s[2 * tp][j] += f;
            ss[2 * tp][j] += f * f;
            s[2 * tp + 1][j] += f2;
            ss[2 * tp + 1][j] += f2 * f2;
          }
        }
      }
    }
  }
  if (!a.stats) return;
#pragma unroll
  for (int kt = 0; kt < KT; ++kt)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float v1 = st_row16_sum(s[kt][j]), v2 = st_row16_sum(ss[kt][j]);
      if ((lane & 15) == 0) {
        red[w][0][st_perm(16 * kt + 4 * (lane >> 4) + j)] = v1;
        red[w][1][st_perm(16 * kt + 4 * (lane >> 4) + j)] = v2;
      }
    }
  __syncthreads();
  if (tid < 2 * K) {
    const int h = tid / K, k = tid - h * K;
    const float v = red[0][h][k] + red[1][h][k] + red[2][h][k] + red[3][h][k];
    atomicAdd(MA_SPREAD(a.stats + ((size_t)(n / a.group_imgs) * 2 + h) * K + k), v);
  }
}

template <int R, int S, int KT>
void stem_go(const StemArgs& a, int blocks, hipStream_t st) {
  hipLaunchKernelGGL((stem_kernel<R, S, KT>), dim3(blocks), dim3(ST_NT), 0, st, a);
}

}  // namespace

// 0: unsupported (R, stride, K) combination
int stem_fwd_launch(StemArgs a, hipStream_t st) {
  if (a.N <= 0 || a.P <= 0 || a.Q <= 0) return 1;
  const int tpi = ((a.P + ST_T - 1) / ST_T) * ((a.Q + ST_T - 1) / ST_T);
  // many more blocks than CU slots (no tail round), the rest as tiles per block (each block
  // stages the weights once and flushes its BN sums once).  A 7x7 stem's weights are 3.5x a
  // 3x3 one's, so it targets 4x fewer blocks; the tiles of an image are split evenly over its
  // blocks (an uneven last block idles its CU); a 32x32 image (4 tiles) is one block when the
  // batch alone fills the CUs.  bench/stem_bench.py, profiles/r5/stem_blocks: ResNet-50 B = 1280
  // 1026 -> 844 us, B = 128 184 -> 125 us, CIFAR B = 320 30.1 -> 26.8 us, VGG unchanged.
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  int tpb = (tpi * a.N) / (a.R > 3 ? 1024 : 4096);
  tpb = tpb < 1 ? 1 : (tpb > tpi ? tpi : tpb);
  if (tpi <= 4 && a.N >= cus) tpb = tpi;
  const int bpi = (tpi + tpb - 1) / tpb;
  tpb = (tpi + bpi - 1) / bpi;
  a.tpb = tpb;
  a.blocks_per_img = (tpi + tpb - 1) / tpb;
  if (a.group_imgs <= 0) a.group_imgs = a.N;
  const int blocks = a.N * a.blocks_per_img;
  const int key = a.R * 100 + a.stride * 10 + a.K / 16;
  switch (key) {
    case 314: stem_go<3, 1, 4>(a, blocks, st); return 1;     // CIFAR ResNet / VGG: 3x3 -> 64
    case 312: stem_go<3, 1, 2>(a, blocks, st); return 1;     // MobileNetV2 (CIFAR): 3x3 -> 32
    case 324: stem_go<3, 2, 4>(a, blocks, st); return 1;
    case 322: stem_go<3, 2, 2>(a, blocks, st); return 1;     // MobileNetV2 (ImageNet): 3x3/2 -> 32
    case 724: stem_go<7, 2, 4>(a, blocks, st); return 1;     // ImageNet ResNet: 7x7/2 -> 64
    default: return 0;
  }
}
