// Fused flat-buffer optimizer.
//
// One launch sweeps the flat fp32 parameter buffer (11.17M elements for ResNet-18), or a
// [start, end) range of whole segments when the step is split (the engine updates the last
// blocks' parameters while earlier blocks are still in backward): Adam (torch.optim.Adam semantics, bias-corrected, L2 weight decay
// folded into the gradient) or SGD with momentum, then -- in the same pass --
// writes the bf16 operand copies the MFMA kernels consume:
//   conv weight (master layout [K][R][S][C]) -> [K][R][S][Cpad] bf16 (fwd/wgrad B)
//                                            -> [C][R][S][K]    bf16 (dgrad B)
// and zeroes the gradient it consumed, so the next backward can accumulate with
// atomics without a separate memset.  The reference does flatten -> all-reduce ->
// divide -> unflatten -> per-tensor Adam -> (cuDNN re-reads fp32 weights); here
// the all-reduce works in place on the same flat gradient and this is the only
// optimizer pass.
//
// Segments are 4-element aligned in the flat buffer, so every thread handles one
// float4 that never straddles two parameters.  Hyper-parameters (lr from the
// cosine schedule) and the step counter live in device memory so the launch is
// graph-capturable and replays with the current values.
#include "common.h"
#include "kernels.h"

namespace {
constexpr int NT = 256;

MA_DEV int find_seg(const OptSeg* s, int n, long long e) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (s[mid].off <= e) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// bf16 [K][R][S][Cpad] forward copy.  The [C][R][S][K] dgrad copy is NOT written
// here (a per-element scatter with stride K would turn every store into a partial
// cache-line update); transpose_weights_kernel produces it tile-by-tile through LDS.
MA_DEV void write_copies(const OptSeg& sg, long long local, float v) {
  if (sg.kind != 1 || local >= sg.numel) return;
  const int rsc = sg.R * sg.S * sg.C;
  const int k = (int)(local / rsc);
  const int rem = (int)(local - (long long)k * rsc);
  const int rs = rem / sg.C, c = rem - rs * sg.C;
  sg.w_krsc[((size_t)k * sg.R * sg.S + rs) * sg.Cpad + c] = f2bf(v);
}

// One 64(k) x 64(c) tile of one (segment, r*S+s) per workgroup: coalesced 2-byte reads
// along c from the KRSC copy, LDS transpose, coalesced writes along k to CRSK.  The tile
// holds one value per dword (bf16 -> fp32 -> bf16 is exact) with a 65-dword row stride, so
// the column read tile[tx][r] hits bank (tx + r) mod 64 -- a 2-byte tile with a 65-element
// stride put two lanes in every dword and measured one bank conflict per LDS instruction
// (SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS = 1.0, profiles/pmc_step_r1f.txt).  Conflicts are now 0
// but the kernel time is unchanged (20.6 -> 21.0 us): it is bound by its 2-byte global
// accesses, so the next step is 16-byte (bf16x8) loads and stores.
__global__ __launch_bounds__(256) void transpose_weights_kernel(const OptSeg* segs,
                                                                const int* jobs) {
  __shared__ float tile[64][65];
  const int* j = jobs + blockIdx.x * 4;
  const OptSeg sg = segs[j[0]];
  const int rs = j[1], k0 = j[2], c0 = j[3];
  const int RS = sg.R * sg.S;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int k = k0 + r, c = c0 + tx;
    tile[r][tx] = (k < sg.K && c < sg.C) ? bf2f(sg.w_krsc[((size_t)k * RS + rs) * sg.Cpad + c]) : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int c = c0 + r, k = k0 + tx;
    if (c < sg.C && k < sg.K) sg.w_crsk[((size_t)c * RS + rs) * sg.K + k] = f2bf(tile[tx][r]);
  }
}

// Adam / AdamW / SGD-momentum on 4 consecutive elements (the flat layout keeps segments
// 4-aligned, so a float4 never straddles two parameters)
struct OptHyper {
  float lr, b1, b2, eps, wd, step_size, rbc2;
  bool first;
};

MA_DEV OptHyper opt_hyper(const OptArgs& a) {
  OptHyper h;
  h.lr = a.hyper[0];
  h.b1 = a.hyper[1];
  h.b2 = a.hyper[2];
  h.eps = a.hyper[3];
  h.wd = a.hyper[4];
  const float t = (float)(*a.step);
  h.step_size = h.lr / (1.f - __powf(h.b1, t));
  h.rbc2 = rsqrtf(1.f - __powf(h.b2, t));
  h.first = *a.step <= 1;
  return h;
}

MA_DEV float4 opt_update4(const OptArgs& a, const OptHyper& h, long long e) {
  float4 p = *(const float4*)(a.p + e);
  float4 g = *(const float4*)(a.g + e);
  float4 m = *(const float4*)(a.m + e);
  float pv[4] = {p.x, p.y, p.z, p.w}, gv[4] = {g.x, g.y, g.z, g.w}, mv[4] = {m.x, m.y, m.z, m.w};
  if (a.algo == 0 || a.algo == 2) {
    float4 v = *(const float4*)(a.v + e);
    float vv[4] = {v.x, v.y, v.z, v.w};
    const bool decoupled = a.algo == 2;   // AdamW: p *= 1 - lr*wd before the Adam update
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float gk = gv[k];
      if (decoupled) pv[k] *= 1.f - h.lr * h.wd;
      else if (h.wd != 0.f) gk += h.wd * pv[k];
      mv[k] = h.b1 * mv[k] + (1.f - h.b1) * gk;
      vv[k] = h.b2 * vv[k] + (1.f - h.b2) * gk * gk;
      const float denom = sqrtf(vv[k]) * h.rbc2 + h.eps;
      pv[k] -= h.step_size * mv[k] / denom;
    }
    *(float4*)(a.v + e) = make_float4(vv[0], vv[1], vv[2], vv[3]);
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float gk = gv[k];
      if (h.wd != 0.f) gk += h.wd * pv[k];
      mv[k] = h.first ? gk : h.b1 * mv[k] + gk;
      pv[k] -= h.lr * mv[k];
    }
  }
  const float4 pn = make_float4(pv[0], pv[1], pv[2], pv[3]);
  *(float4*)(a.p + e) = pn;
  *(float4*)(a.m + e) = make_float4(mv[0], mv[1], mv[2], mv[3]);
  if (a.zero_grad) *(float4*)(a.g + e) = make_float4(0.f, 0.f, 0.f, 0.f);
  return pn;
}

MA_DEV void write_krsc4(const OptSeg& sg, long long local, const float4& pn) {
  const float pv[4] = {pn.x, pn.y, pn.z, pn.w};
  if ((sg.C & 3) == 0 && local + 3 < sg.numel) {  // 4 consecutive channels: one 8-B store
    const int rsc = sg.R * sg.S * sg.C;
    const int k = (int)(local / rsc);
    const int rem = (int)(local - (long long)k * rsc);
    const int rs = rem / sg.C, c = rem - rs * sg.C;
    bf16x4 b;
#pragma unroll
    for (int q = 0; q < 4; ++q) b[q] = f2bf(pv[q]);
    *(bf16x4*)(sg.w_krsc + ((size_t)k * sg.R * sg.S + rs) * sg.Cpad + c) = b;
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) write_copies(sg, local + q, pv[q]);
  }
}

__global__ __launch_bounds__(NT) void optimizer_kernel(OptArgs a) {
  const long long i4 = (long long)blockIdx.x * NT + threadIdx.x;
  const long long e = a.start + i4 * 4;
  if (e >= a.total) return;
  const int si = find_seg(a.segs, a.nsegs, e);
  const OptSeg sg = a.segs[si];
  const float4 pn = opt_update4(a, opt_hyper(a), e);
  if (sg.kind == 1) write_krsc4(sg, e - sg.off, pn);
}

// The whole step in ONE launch, with the dgrad weight copy produced from the update itself
// (no separate transpose kernel re-reading the bf16 forward copy with 2-byte accesses):
//   blocks [0, njobs)  : one 64(k) x 64(c) tile of one (conv segment, r*S+s) each -- 16 rows of
//                        4 float4 per thread, coalesced 256-B rows of p/g/m/v, the bf16 [K][R][S]
//                        [Cpad] copy from registers, and the [C][R][S][K] copy through an LDS
//                        transpose written as 16-byte chunks of 8 k;
//   blocks [njobs, ..) : every other element (BN / fc / conv segments the tiles do not cover),
//                        float4 per thread over the concatenated ranges `ew` ([n][2] = start,
//                        numel; prefix sums in float4 units in `ewp`).
__global__ __launch_bounds__(NT) void optimizer_fused_kernel(OptArgs a, const int* jobs, int njobs,
                                                             const long long* ew,
                                                             const long long* ewp, int new_) {
  const OptHyper h = opt_hyper(a);
  if ((int)blockIdx.x < njobs) {
    // pitch 65 plus column XOR (row >> 3) * 4: the transposed reads (8 lanes down a column,
    // 8 rows apart, 4 columns) hit 32 distinct banks; the row writes stay 2-way (free for b32)
    __shared__ float tile[64][65];
    auto tcol = [](int r, int c) { return c ^ (((r >> 3) & 7) << 2); };
    const int* j = jobs + blockIdx.x * 4;
    const OptSeg sg = a.segs[j[0]];
    const int rs = j[1], k0 = j[2], c0 = j[3];
    const int RS = sg.R * sg.S;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;   // 16 float4 columns x 16 rows
    const int c = c0 + tx * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = ty + 16 * i, k = k0 + r;
      float4 pn = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k < sg.K && c < sg.C) {                 // host: C % 4 == 0, so c < C => c + 3 < C
        const long long local = ((long long)k * RS + rs) * sg.C + c;
        pn = opt_update4(a, h, sg.off + local);
        bf16x4 b;
        b[0] = f2bf(pn.x);
        b[1] = f2bf(pn.y);
        b[2] = f2bf(pn.z);
        b[3] = f2bf(pn.w);
        *(bf16x4*)(sg.w_krsc + ((size_t)k * RS + rs) * sg.Cpad + c) = b;
      }
      tile[r][tcol(r, tx * 4 + 0)] = pn.x;
      tile[r][tcol(r, tx * 4 + 1)] = pn.y;
      tile[r][tcol(r, tx * 4 + 2)] = pn.z;
      tile[r][tcol(r, tx * 4 + 3)] = pn.w;
    }
    __syncthreads();
    // [C][R][S][K]: row (c, rs) holds k contiguous -> 8 chunks of 8 k per 64-k tile row
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = threadIdx.x + NT * i;         // 512 chunks = 64 c x 8
      const int cr = q >> 3, kc = (q & 7) * 8;
      const int cc = c0 + cr, kk = k0 + kc;
      if (cc < sg.C && kk < sg.K) {
        bf16x8 o;
#pragma unroll
        for (int t = 0; t < 8; ++t) o[t] = f2bf(tile[kc + t][tcol(kc + t, cr)]);
        bf16* dst = sg.w_crsk + ((size_t)cc * RS + rs) * sg.K + kk;
        if (kk + 8 <= sg.K && (sg.K & 7) == 0) {
          *(bf16x8*)dst = o;
        } else {
          for (int t = 0; t < 8 && kk + t < sg.K; ++t) dst[t] = o[t];
        }
      }
    }
    return;
  }
  // elementwise remainder
  const long long v4 = (long long)(blockIdx.x - njobs) * NT + threadIdx.x;
  if (v4 >= ewp[new_]) return;
  int lo = 0, hi = new_ - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (ewp[mid] <= v4) lo = mid;
    else hi = mid - 1;
  }
  const long long e = ew[2 * lo] + (v4 - ewp[lo]) * 4;
  const float4 pn = opt_update4(a, h, e);
  const OptSeg sg = a.segs[find_seg(a.segs, a.nsegs, e)];
  if (sg.kind == 1) write_krsc4(sg, e - sg.off, pn);
}

__global__ __launch_bounds__(NT) void pack_kernel(const float* p, const OptSeg* segs, int nsegs,
                                                  long long total) {
  const long long e = (long long)blockIdx.x * NT + threadIdx.x;
  if (e >= total) return;
  const OptSeg sg = segs[find_seg(segs, nsegs, e)];
  write_copies(sg, e - sg.off, p[e]);
}

// start of a train step: bump the Adam step counter and zero the step's BN-statistics and
// BN-backward-sum arenas (one launch instead of one kernel + two memsets on the critical path)
__global__ __launch_bounds__(256) void step_begin_kernel(int64_t* ctrl, float* z0, int n0,
                                                         float* z1, int n1) {
  if (blockIdx.x == 0 && threadIdx.x == 0) ctrl[2] += 1;
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int stride = gridDim.x * 256;
  for (int j = i; j < n0; j += stride) z0[j] = 0.f;
  for (int j = i; j < n1; j += stride) z1[j] = 0.f;
}
}  // namespace

void optimizer_launch(const OptArgs& a, hipStream_t st) {
  if (a.total <= a.start) return;
  const long long n4 = (a.total - a.start + 3) / 4;
  hipLaunchKernelGGL(optimizer_kernel, dim3((unsigned)((n4 + NT - 1) / NT)), dim3(NT), 0, st, a);
}

void optimizer_fused_launch(const OptArgs& a, const int* jobs, int njobs, const long long* ew,
                            const long long* ewp, int new_, long long ew4, hipStream_t st) {
  const long long blocks = njobs + (ew4 + NT - 1) / NT;
  if (blocks > 0)
    hipLaunchKernelGGL(optimizer_fused_kernel, dim3((unsigned)blocks), dim3(NT), 0, st, a, jobs,
                       njobs, ew, ewp, new_);
}

void pack_weights_launch(const float* p, const OptSeg* segs, int nsegs, long long total,
                         hipStream_t st) {
  hipLaunchKernelGGL(pack_kernel, dim3((unsigned)((total + NT - 1) / NT)), dim3(NT), 0, st, p, segs,
                     nsegs, total);
}

void transpose_weights_launch(const OptSeg* segs, const int* jobs, int njobs, hipStream_t st) {
  if (njobs > 0)
    hipLaunchKernelGGL(transpose_weights_kernel, dim3(njobs), dim3(256), 0, st, segs, jobs);
}

void step_begin_launch(int64_t* ctrl, float* z0, int n0, float* z1, int n1, hipStream_t st) {
  const int n = n0 > n1 ? n0 : n1;
  int blocks = (n + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 256 ? 256 : blocks);
  hipLaunchKernelGGL(step_begin_kernel, dim3(blocks), dim3(256), 0, st, ctrl, z0, n0, z1, n1);
}
