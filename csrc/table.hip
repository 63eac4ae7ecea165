// Global importance table resident in HBM (`util.py:94-160` Groupwise_Sampler).
//
// One float importance and one int32 group stamp per dataset sample (50k CIFAR = 400 KB,
// 1.28M ImageNet = 10 MB -- trivially resident in 288 GB of HBM, so the table is never
// copied to the host).  The reference re-normalises the current group on the CPU for every
// single draw (`util.py:144-152`, O(N) numpy work per sample); here a draw batch costs three
// small launches, all graph-capturable:
//
//   table_partial : grid-stride over the table in TSEG-entry segments (one workgroup per
//                   segment, 8 entries/thread with 16B loads): masked sum and count per segment.
//   table_prep    : one workgroup: group mean, per-segment weights  w_b = sum_b + cnt_b*mean
//                   (the reference's alpha=1 smoothing  w = imp + mean(imp)), exclusive fp64
//                   scan -> segment prefix, snapshot + bump of the device draw counter.
//   table_draw    : one wave per draw: Philox uniform -> binary search over segment prefix ->
//                   the wave sums 64 lane-contiguous 32-entry slices, wave prefix scan picks the
//                   slice, the owning lane walks its slice.  O(log N + 64) per draw, no host.
//
// Two-level inverse CDF instead of a global alias table: the table changes between draw
// batches (the reference applies updates live, `util.py:141`), so a build has to be cheap --
// one read pass -- which a parallel alias construction (split/pack of light/heavy items) is
// not.  The pool sampler (is_sample, P<=16k) does use an LDS alias table.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int TSEG = 2048;                 // entries per segment (= 64 lanes x 32)
constexpr int TPB = 256;                   // threads per partial block -> 8 entries each

__global__ __launch_bounds__(TPB) void table_scatter_kernel(TableScatterArgs a) {
  const int i = blockIdx.x * TPB + threadIdx.x;
  if (i >= a.n) return;
  const int pos = a.index ? a.index[i] : a.start + i;
  if (pos < 0 || pos >= a.N) return;
  a.imp[pos] = a.losses[i];
  a.grp[pos] = a.stamp ? (int)a.stamp[0] : a.gi;
}

__global__ __launch_bounds__(TPB) void table_partial_kernel(const float* imp, const int* grp, int N,
                                                            int gi, const int64_t* gi_dev,
                                                            float2* part) {
  __shared__ float red[16];
  const int g = gi_dev ? (int)gi_dev[0] : gi;
  const int base = blockIdx.x * TSEG + threadIdx.x * 8;
  float s = 0.f, c = 0.f;
  if (base + 8 <= N) {
    const f32x4 i0 = *(const f32x4*)(imp + base), i1 = *(const f32x4*)(imp + base + 4);
    const int4 g0 = *(const int4*)(grp + base), g1 = *(const int4*)(grp + base + 4);
    const float iv[8] = {i0.x, i0.y, i0.z, i0.w, i1.x, i1.y, i1.z, i1.w};
    const int gv[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (gv[k] == g) { s += iv[k]; c += 1.f; }
  } else {
    for (int k = base; k < min(N, base + 8); ++k)
      if (grp[k] == g) { s += imp[k]; c += 1.f; }
  }
  s = block_sum(s, red);
  c = block_sum(c, red);
  if (threadIdx.x == 0) part[blockIdx.x] = make_float2(s, c);
}

__global__ __launch_bounds__(1024) void table_prep_kernel(const float2* part, int nseg,
                                                          double* prefix, TableScalars* sc,
                                                          int64_t* counter) {
  __shared__ double dsum[1024];
  __shared__ float red[16];
  const int tid = threadIdx.x;
  const int per = (nseg + 1023) / 1024;
  const int b0 = min(nseg, tid * per), b1 = min(nseg, b0 + per);
  float s = 0.f, c = 0.f;
  for (int b = b0; b < b1; ++b) { s += part[b].x; c += part[b].y; }
  const float ts = block_sum(s, red), tc = block_sum(c, red);
  const float mean = tc > 0.f ? ts / tc : 0.f;
  double local = 0.0;
  for (int b = b0; b < b1; ++b) local += (double)part[b].x + (double)part[b].y * mean;
  dsum[tid] = local;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {       // Hillis-Steele inclusive scan (fp64)
    const double add = tid >= off ? dsum[tid - off] : 0.0;
    __syncthreads();
    dsum[tid] += add;
    __syncthreads();
  }
  double run = tid > 0 ? dsum[tid - 1] : 0.0;
  for (int b = b0; b < b1; ++b) {
    prefix[b] = run;
    run += (double)part[b].x + (double)part[b].y * mean;
  }
  if (tid == 1023) prefix[nseg] = dsum[1023];
  if (tid == 0) {
    sc->mean = mean;
    sc->count = tc;
    sc->total = dsum[1023];
    const int64_t ctr = counter ? counter[0] : 0;
    sc->counter = ctr;
    if (counter) counter[0] = ctr + 1;
  }
}

MA_DEV float wave_incl_scan(float v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

__global__ __launch_bounds__(256) void table_draw_kernel(const float* imp, const int* grp, int N,
                                                         int gi, const int64_t* gi_dev,
                                                         const double* prefix, int nseg,
                                                         const TableScalars* sc, int ndraw,
                                                         uint32_t seed, int64_t* out,
                                                         int* out32) {
  const int lane = threadIdx.x & 63;
  const int d = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (d >= ndraw) return;
  const int g = gi_dev ? (int)gi_dev[0] : gi;
  const double total = sc->total;
  const float mean = sc->mean;
  const uint64_t ctr = (uint64_t)sc->counter;
  if (!(total > 0.0)) {                     // empty group: nothing to draw from
    if (lane == 0) {
      if (out) out[d] = -1;
      if (out32) out32[d] = -1;
    }
    return;
  }
  const u32x4 r = philox4x32(u32x4{(uint32_t)ctr, (uint32_t)(ctr >> 32), (uint32_t)d, 0x7ab1e5u},
                             seed, 0x1B873593u);
  const double u01d = ((double)r.x + (double)r.y * 4294967296.0) * (1.0 / 18446744073709551616.0);
  const double u = fmin(u01d * total, total * (1.0 - 1e-12));
  // largest segment b with prefix[b] <= u  (skips zero-weight segments, see header)
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (prefix[mid] <= u) lo = mid;
    else hi = mid - 1;
  }
  const int seg = lo;
  const float rem = (float)(u - prefix[seg]);
  const int base = seg * TSEG + lane * 32;
  float ls = 0.f;
  for (int k = 0; k < 32; k += 4) {
    const int e = base + k;
    if (e + 4 <= N) {
      const f32x4 iv = *(const f32x4*)(imp + e);
      const int4 gv = *(const int4*)(grp + e);
      ls += (gv.x == g ? iv.x + mean : 0.f) + (gv.y == g ? iv.y + mean : 0.f) +
            (gv.z == g ? iv.z + mean : 0.f) + (gv.w == g ? iv.w + mean : 0.f);
    } else {
      for (int q = e; q < min(N, e + 4); ++q)
        if (grp[q] == g) ls += imp[q] + mean;
    }
  }
  const float incl = wave_incl_scan(ls, lane);
  const uint64_t hit = __ballot(incl > rem && ls > 0.f);
  const uint64_t nz = __ballot(ls > 0.f);
  // fp32 re-summation can disagree with the fp64 prefix by an ulp: fall back to the last
  // non-empty slice of the segment
  const int owner = hit ? __ffsll((long long)hit) - 1 : 63 - __clzll((long long)nz);
  if (lane != owner) return;
  float run = incl - ls;
  int pick = -1, last = -1;
  for (int q = base; q < min(N, base + 32); ++q) {
    if (grp[q] != g) continue;
    last = q;
    run += imp[q] + mean;
    if (run > rem) { pick = q; break; }
  }
  if (pick < 0) pick = last;
  if (out) out[d] = pick;
  if (out32) out32[d] = pick;
}

// Native groupwise step (engine sampler='groupwise'): the drawn table positions -> pool slots
// of the current contiguous slice (slot = (pos - slice start) mod Ns; the slice is exactly the
// current group) and unbiased importance weights  w = n_group * p = n_group (imp + mean) / total
// (the pool sampler's N*p convention: the train loss divides by w).  meters[3] gets the group's
// mean importance (the pool-mean slot).
__global__ __launch_bounds__(256) void table_weights_kernel(const int* pos, int ndraw,
                                                            const float* imp,
                                                            const TableScalars* sc,
                                                            const int* pool_index, int Ns, int P,
                                                            int* idx, float* isw, float* meters) {
  const int d = blockIdx.x * 256 + threadIdx.x;
  const float mean = sc->mean, cnt = sc->count;
  const double total = sc->total;
  if (d == 0 && meters) meters[3] = mean;
  if (d >= ndraw) return;
  const int q = pos[d];
  if (q < 0 || !(total > 0.0)) {          // empty group (cannot happen after a scatter): slot 0
    idx[d] = 0;
    isw[d] = 1.f;
    return;
  }
  int slot = q - pool_index[0];
  slot = slot < 0 ? slot + Ns : slot;
  idx[d] = slot < P ? slot : P - 1;
  isw[d] = (float)((double)cnt * ((double)imp[q] + (double)mean) / total);
}

}  // namespace

void table_weights_launch(const int* pos, int ndraw, const float* imp, const void* sc,
                          const int* pool_index, int Ns, int P, int* idx, float* isw,
                          float* meters, hipStream_t st) {
  hipLaunchKernelGGL(table_weights_kernel, dim3((ndraw + 255) / 256), dim3(256), 0, st, pos, ndraw,
                     imp, (const TableScalars*)sc, pool_index, Ns, P, idx, isw, meters);
}

int table_num_segments(int N) { return (N + TSEG - 1) / TSEG; }

void table_scatter_launch(const TableScatterArgs& a, hipStream_t st) {
  if (a.n <= 0) return;
  hipLaunchKernelGGL(table_scatter_kernel, dim3((a.n + TPB - 1) / TPB), dim3(TPB), 0, st, a);
}

void table_sample_launch(const TableSampleArgs& a, hipStream_t st) {
  const int nseg = table_num_segments(a.N);
  hipLaunchKernelGGL(table_partial_kernel, dim3(nseg), dim3(TPB), 0, st, a.imp, a.grp, a.N, a.gi,
                     a.gi_dev, a.part);
  hipLaunchKernelGGL(table_prep_kernel, dim3(1), dim3(1024), 0, st, a.part, nseg, a.prefix, a.sc,
                     a.counter);
  if (a.ndraw > 0)
    hipLaunchKernelGGL(table_draw_kernel, dim3((a.ndraw + 3) / 4), dim3(256), 0, st, a.imp, a.grp,
                       a.N, a.gi, a.gi_dev, a.prefix, nseg, a.sc, a.ndraw, a.seed, a.out,
                       a.out32);
}
