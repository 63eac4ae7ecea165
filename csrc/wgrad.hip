// Weight-gradient implicit GEMM on MFMA (gfx950).
//
//   dW[k][(r,s,c)] = sum_pixels dy[pix][k] * x[n, p*stride-pad+r, q*stride-pad+s, c]
//
// (the `loss.backward()` of `pytorch_collab.py:148` for every conv).
// The reduction runs over pixels, which is the STRIDED axis of both NHWC
// operands, so tiles are staged in LDS as [pixel][channel] rows (16-byte
// coalesced loads along channels) and the MFMA fragments -- which need 8
// consecutive reduction elements per lane -- are read with the gfx950 hardware
// transpose `ds_read_b64_tr_b16`: one instruction delivers, per 16-lane group, a
// 4-pixel x 16-channel block column-major.  Two reads give the 8 k-values of a
// v_mfma_f32_16x16x32_bf16 operand.
//
// LDS rows are padded to (cols+16) bf16 so a row shifts 8 banks; the pixel
// order inside a 32-deep k-step is permuted identically for both operands
// (element j of lane-group g <- pixel 16*(j>>2) + 4*g + (j&3)) so each 32-lane
// half reads 8 consecutive rows: conflict-free tr reads.  The permutation is a
// relabelling of the summation index, so the result is unchanged.
//
// Split-K over pixels (gridDim.y) either reduces through a slab (the last split to arrive
// on a tile sums the partial tiles and stores: the large-pixel-count convs, where the split
// count is high) or accumulates with fp32 atomics into the flat gradient buffer; without
// splitting it stores.  The output is written in the
// engine's master layout [K][R][S][Creal] (channel padding dropped).

#include "wgrad_body.h"

namespace {
using namespace wgb;
constexpr int NT = WG_NT;
constexpr int BKP = WG_BKP;

template <int BM, int BN>
__global__ __launch_bounds__(NT, 2) void wgrad_kernel(const bf16* __restrict__ dy,
                                                       const bf16* __restrict__ x, WgradGeom g,
                                                       float* __restrict__ dw, int ptiles_per_split) {
  __shared__ __attribute__((aligned(16))) bf16 smem[WgSmem<BM, BN>::STAGE * 2];
  wgrad_body<BM, BN>(dy, x, g, dw, ptiles_per_split, smem, blockIdx.x, blockIdx.y, gridDim.y);
}

template <int BM, int BN>
void wlaunch(const bf16* dy, const bf16* x, const WgradGeom& g, float* dw, int splits,
             hipStream_t st) {
  int gx, per, gy;
  wg_grid(g, BM, BN, splits, gx, per, gy);
  WgradGeom gg = g;
  if (gx > WG_SEM_INTS) gg.slab = nullptr;   // counters would not fit: atomic splits
  hipLaunchKernelGGL((wgrad_kernel<BM, BN>), dim3(gx, gy), dim3(NT), 0, st, dy, x, gg, dw, per);
}
}  // namespace

__device__ __attribute__((aligned(16))) bf16 g_wg_zero[64];

void wgrad_launch(const bf16* dy, const bf16* x, const WgradGeom& g_in, float* dw, int bm, int bn,
                  int splits, hipStream_t st) {
  static const bf16* zp = nullptr;
  if (!zp) {
    void* p = nullptr;
    (void)hipGetSymbolAddress(&p, HIP_SYMBOL(g_wg_zero));
    zp = (const bf16*)p;
  }
  WgradGeom g = g_in;
  g.zero = zp;
  if (bm == 128 && bn == 128) return wlaunch<128, 128>(dy, x, g, dw, splits, st);
  if (bm == 128 && bn == 64) return wlaunch<128, 64>(dy, x, g, dw, splits, st);
  if (bm == 64 && bn == 128) return wlaunch<64, 128>(dy, x, g, dw, splits, st);
  return wlaunch<64, 64>(dy, x, g, dw, splits, st);
}
