// Host-visible parameter blocks for the implicit-GEMM conv kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

typedef __bf16 bf16;

// A-operand gather geometry.  "S*" = the tensor A is gathered from (NHWC), "R*" =
// the spatial dims the GEMM rows enumerate.  forward: S = input x, R = output (P,Q);
// dgrad (trans): S = dy, R = input (H,W).
struct ConvGeom {
  int SH, SW, SC;    // source spatial dims and (padded) channels
  int RP, RQ;        // row-space spatial dims
  int R, S, stride, pad;
  int Kc;            // reduction length in 8-element chunks = R*S*SC/8
  int Ncols;         // GEMM N (output channels)
  int M;             // GEMM M = images * RP * RQ
  const bf16* zero;  // 16-byte zero page for padding taps (set by the launcher; kernel arg -> SGPR)
  // stride-2 dgrad parity class (dgrad_s2_launch): the class is a stride-1 FORWARD gather of dy
  // whose virtual tap (r', s') reads the real weight tap (trb - 2 r', tsb - 2 s') of a [C][R][S][K]
  // weight with row stride ldb; trb < 0: plain (B chunk = k chunk, row stride Kc * 8)
  int ldb = 0;
  int trb = -1, tsb = 0, tS = 0;
};

// BN-backward sums are kept as SUMS_R replicas [SUMS_R][3][C]: a producer block adds into
// replica (its tile / block index % SUMS_R) and bn_bwd_apply, their one consumer, sums the
// replicas when it loads them.  Every block adding into ONE [3][C] row serialised at the memory
// side (bench/stats_cost.py: the ResNet-18 layer-1 dgrad+wgrad pair 32.8 us with the fused sums,
// 20.5 without).
constexpr int SUMS_R = 8;

struct EpiParams {
  bf16* out;          // [M][ldo] bf16
  int ldo;
  const float* bias;  // [N] or null
  float* stats;       // BN sums: [G][2][stats_ld] (sum, sumsq) or null
  int stats_ld;
  int group_rows;     // rows per ghost-BN group (>= BM; a tile straddles at most one boundary)
  int accumulate;     // out += result
  float* slab;        // split-K workspace (set by the launcher's caller when splits > 1)
  // Fused BN-backward reduction over the FINAL output values g (a gradient wrt the output of
  // BN[+BN2]+act, e.g. dgrad of the next conv): dz = g * act'(bw_out);
  //   bw_sums[0][c] += sum dz,  [1][c] += sum dz*xhat(bw_y),  [2][c] += sum dz*xhat(bw_y2)
  // (the reduce pass of bn_bwd; bn_bwd then only applies).  Same [M][ldo] layout as out.
  const bf16* bw_out;
  const bf16* bw_y;
  const float* bw_stats;   // [2][ldo] batch sum, sumsq of bw_y
  const bf16* bw_y2;       // optional shortcut BN sharing dz
  const float* bw_stats2;
  float* bw_sums;          // [SUMS_R][3][ldo] replicas (SUMS_R above) or null (feature off)
  float bw_inv_count, bw_eps;
  int bw_act;
  // output row remap of a stride-2 dgrad parity class: GEMM row (n, i, j) over rm_hc x rm_wc is
  // the output pixel (n, 2i + rm_ph, 2j + rm_pw) of an rm_h x rm_w image; rm_hc == 0: identity
  int rm_hc = 0, rm_wc = 0, rm_h = 0, rm_w = 0, rm_ph = 0, rm_pw = 0;
};

// Forward-only A-operand prologue: the conv reads the PRODUCING conv's raw output y and applies
// that layer's BatchNorm + activation per input channel while staging the tile,
//   a = act(y * scale + shift),  scale = gamma * rsqrt(var + eps),  shift = beta - mean * scale
// (batch / ghost-group statistics from the producer's epilogue sums, or running statistics),
// so the normalised activation never makes its own HBM round trip.  Padding taps stay zero (the
// zero lives in activation space).  ``keep`` (optional) receives the activation as well: the
// chunk loaded at tap ``keep_tap`` of a stride-1 "same" conv is exactly the output pixel's own
// input pixel, so the N-tile-0 blocks write every element of ``a`` once (train mode: backward
// needs it).
struct ProParams {
  const float* stats;   // [G][2][SC] (sum, sumsq) of y per stat group, or null (running stats)
  const float* rmean;   // running mean / var (used when stats == null)
  const float* rvar;
  const float* gamma;
  const float* beta;
  bf16* keep;           // [SH*SW*images][SC] activation write-back, or null
  int group_rows;       // OUTPUT rows per stat group (a multiple of the tile's BM)
  float inv_count;      // 1 / y-pixels per stat group
  float eps;
  int act;              // 0 none, 1 relu, 2 relu6
  int keep_tap;         // r*S + s of the tap whose pixel is the output pixel itself
  const bf16* res = nullptr;   // identity residual added before the activation, or null
                               // (a = act(bn(y) + res): a block-final BN feeding the next block)
};

size_t igemm_slab_bytes(const ConvGeom& g, int bm, int bn, int splits);
// pro != null: BN-apply prologue (forward only).
void igemm_launch(const bf16* src, const bf16* wt, const ConvGeom& g, const EpiParams& e, int bm,
                  int bn, int splits, bool trans, hipStream_t st, const ProParams* pro = nullptr);

struct WgradGeom {
  int N, H, W, C;     // input x (C padded), NHWC
  int P, Q, K;        // dy dims (K = output channels)
  int R, S, stride, pad;
  int Creal;          // unpadded input channels (layout of dW)
  const bf16* zero;   // 16-byte zero page (set by the launcher)
  float* slab;        // split-K partial tiles behind WG_SEM_INTS tile counters, or null
                      // (null: the pixel splits add into dW with fp32 atomics)
};
void wgrad_launch(const bf16* dy, const bf16* x, const WgradGeom& g, float* dw, int bm, int bn,
                  int splits, hipStream_t st);

// stride-2 dgrad as four parity classes of input pixels in ONE launch (each class a stride-1
// forward gather of dy over only the taps that reach it: 1/2/2/4 of a 3x3's 9); returns 0 when
// the conv does not qualify (stride 2, 3x3 pad 1 or 1x1 pad 0, dy channels % 64)
int dgrad_s2_launch(const bf16* dy, const bf16* wt, const ConvGeom& g, const EpiParams& e, int bm,
                    int bn, int H, int W, int N, hipStream_t st);

// the pair with the stride-2 class dgrad (dgrad tiles 64 x 64; returns 0 if not instantiated)
int conv_bwd_pair_s2_launch(const bf16* dy, const bf16* wt, const ConvGeom& g, const EpiParams& e,
                            int bm, int bn, int H, int W, int N, const bf16* x,
                            const WgradGeom& wg, float* dw, int wbm, int wbn, int wsplits,
                            hipStream_t st);

// dgrad (TRANS igemm) + wgrad in ONE launch (returns 0 if the tile pair is not instantiated)
int conv_bwd_pair_launch(const bf16* dy, const bf16* wt, const ConvGeom& g, const EpiParams& e,
                         int bm, int bn, int splits, const bf16* x, const WgradGeom& wg, float* dw,
                         int wbm, int wbn, int wsplits, hipStream_t st);

// ---------------------------------------------------------------------------- halo conv
// Forward convolution whose A operand is a HALO TILE in LDS (hconv.hip): a block's output
// tile is IMG whole images or TR whole output rows of one image, so the input it reads for
// one 64-channel slice is a small rectangle, staged into LDS ONCE and read by every tap.
// The persistent / row-step variants can apply the producer's BatchNorm + activation while
// staging (HconvPro; the scoring pass's intra-block BN), so that normalised activation never
// makes a separate HBM round trip.
struct HconvGeom {
  int N, H, W, C;        // input NHWC (C padded to a multiple of 64)
  int P, Q, K;           // output pixels per image and channels
  int R, stride, pad;    // R in {1, 3}
  int IMG, TR;           // tile = IMG images x TR output rows (TR == P when IMG > 1)
  int HT, HWd;           // halo rows / columns per image
  int HWP, HALF;         // LDS pitch (pixels per halo row); stride-2 3x3: even columns first,
                         // odd columns from HALF on (0 otherwise) -- both bank-conflict choices
  int HS, SR;            // input step per halo pixel; halo step per output pixel
  int HPIX;              // halo pixels per tile = IMG * HT * HWP
  int SWA;               // halo chunk swizzle c ^ ((p + SWA * halo_row(p)) & 7); per-tile
                         // kernel only (the persistent / row-step kernels need 0)
  int PGRID;             // persistent kernel: this launch's grid (0: the configured default)
  int chunks_per_split;  // 64-channel input slices per K-split
  const bf16* zero;      // 16-byte zero page (set by the launcher)
};

struct HconvPro {
  int mode;              // 0 plain input, 1 act(bn(y)) applied in the halo staging
  const float* stats;    // [G][2][C] batch / ghost-group sums of y, or null -> running stats
  const float* rmean;
  const float* rvar;
  const float* gamma;
  const float* beta;
  int group_imgs;        // images per statistics group
  float inv_count;       // 1 / pixels per statistics group
  float eps;
  int act;               // 0 none, 1 relu, 2 relu6
  int coef_tab = 0;      // (launcher-set) row-step kernel: BN coefficients from an LDS table
};

// returns 0 when (bm, bn) is not instantiated
// ---------------------------------------------------------------------------- pointwise GEMM
// 1x1 convolution as a persistent LDS-DMA-pipelined GEMM (pgemm.hip): OUT[M][ldo] (bf16) =
// A[rows][K] . B[N][K]^T with optional ghost-BN statistics of OUT.  stride != 1: A row of output
// pixel m = (n, p, q) is n*H*W + p*stride*W + q*stride (1x1 stride-2 shortcut convs).
struct PgemmArgs {
  const bf16* a;
  const bf16* b;
  bf16* out;
  float* stats;            // [G][2][stats_ld] (sum, sumsq) or null
  int M, N, K, ldo, stats_ld, group_rows;
  unsigned a_bytes, b_bytes, out_bytes;   // buffer-resource ranges (< 4 GB)
  int H, W, P, Q, stride;
};
// Input prologue of the pointwise GEMM: A = act(bn(y) [+ res]) applied in LDS to each
// operand tile as it lands (once per tile, by the thread whose DMA brought it), from per-group
// scale / shift coefficients that a small kernel derives from the producer's statistics into
// ``coef`` ([G][2][K], launched by pgemm_launch).  ``keep`` (optional) receives the activation:
// the N-tile-0 tiles write each transformed chunk once.  Stride-1 convs only.
struct PgemmPro {
  int mode;                // 0 none, 1 act(bn(y)), 2 act(bn(y) + res)
  const float* stats;      // [G][2][K] producer sums (sum, sumsq) per group, or null: running
  const float* rmean;
  const float* rvar;
  const float* gamma;
  const float* beta;
  float inv_count, eps;
  int act;                 // 0 none, 1 relu, 2 relu6
  int group_rows;          // input rows per statistics group (>= 256, or the whole batch)
  int G;                   // statistics groups (1 with running statistics)
  float* coef;             // workspace [G][2][K]
  const bf16* res;         // mode 2: residual [rows][K]
  bf16* keep;              // optional activation output [rows][K]
  unsigned res_bytes, keep_bytes, coef_bytes;
};
// bn in {64, 128, 256}; grid <= 0: one block per CU.  Returns 0 when unsupported.
int pgemm_launch(const PgemmArgs& g, int bn, int grid, hipStream_t st, const PgemmPro* pro = nullptr);
// Narrow-input (K <= 128) stride-1 1x1 conv with the whole A panel (128 rows x K) resident in
// LDS and normalised once for all N-tiles (pwconv.hip); mode-1 prologue only.  0: unsupported.
int pwconv_launch(const PgemmArgs& g, hipStream_t st, const PgemmPro* pro = nullptr);

int hconv_launch(const bf16* src, const bf16* wt, const HconvGeom& g, const EpiParams& e,
                 const HconvPro& pro, int bm, int bn, int splits, hipStream_t st);
const bf16* conv_zero_page();
