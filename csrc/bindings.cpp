// Python bindings for the mercury_amd HIP kernels.
//
// Deliberately thin: tensors cross the boundary as raw device addresses (int)
// plus the caller's hipStream_t, so this translation unit needs only pybind11 and
// the HIP runtime -- no PyTorch headers -- and builds in seconds.  All shape,
// dtype, device and contiguity validation happens in mercury_amd/ops/*.py, which
// also fails loudly if this extension is missing on a GPU machine.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "kernels.h"

int igemm_read_stamps(unsigned long long* host, int n);
int conv_bwd_pair_sc_launch(const bf16* dyA, const bf16* wtA, const ConvGeom& gA_in,
                            const EpiParams& eA_in, int bm, int bn, int splits, const bf16* xA,
                            const WgradGeom& wgA_in, float* dwA, int wbm, int wbn, int wsplits,
                            const bf16* dyB, const bf16* wtB, const ConvGeom& gtB,
                            const EpiParams& eB_in, int HB, int WB, int NB, const bf16* xB,
                            const WgradGeom& wgB_in, float* dwB, int wsplitsB, hipStream_t st);
int igemm_dual_launch(const bf16* srcA, const bf16* wtA, const ConvGeom& gA, const EpiParams& eA,
                      int splitsA, const bf16* srcB, const bf16* wtB, const ConvGeom& gB,
                      const EpiParams& eB, int splitsB, int bm, int bn, hipStream_t st);
int hconv_read_stamps(unsigned long long* host, int n);
void hconv_configure(int grid, int waves, int wm8);
// native RCCL communicator (comm.hip)
std::string comm_unique_id();
uintptr_t comm_init(const std::string& id_bytes, int rank, int nranks);
void comm_destroy(uintptr_t c);
void comm_allreduce(uintptr_t c, uintptr_t buf, long long count, int dtype, int avg, uintptr_t st);
void comm_allgather(uintptr_t c, uintptr_t send, uintptr_t recv, long long count, int dtype,
                    uintptr_t st);
void comm_broadcast(uintptr_t c, uintptr_t buf, long long count, int dtype, int root, uintptr_t st);
void comm_ring_allreduce(uintptr_t c, uintptr_t buf, long long count, uintptr_t work, int avg,
                         uintptr_t st);
void add_f32(float* dst, const float* src, long long n, hipStream_t s);
// direct-xGMI two-shot all-reduce (xgmi.hip)
void xgmi_pack(const float* src, void* xbuf, long long n, int bf, hipStream_t st);
void xgmi_reduce_scatter(const void* const* peers, int W, int rank, long long n, int bf,
                         float scale, hipStream_t st);
void xgmi_all_gather(const void* const* peers, int W, long long n, int bf, float* dst,
                     hipStream_t st);
int xgmi_max_ranks();
void xgmi_barrier(const void* const* flag_areas, int W, int rank, unsigned* epoch,
                  double timeout_s, int* err, hipStream_t st);
int xgmi_flag_bytes();
std::string xgmi_ipc_handle(uintptr_t ptr);
uintptr_t xgmi_ipc_open(const std::string& handle);
uintptr_t xgmi_malloc(long long bytes);
void xgmi_free(uintptr_t p);
void xgmi_ipc_close(uintptr_t p);
void order_check_launch(int* o, int slot, int ref, int mult, int add, int ge, int tick, int at,
                        hipStream_t st);

namespace py = pybind11;

template <typename T>
static T* P(uintptr_t v) { return reinterpret_cast<T*>(v); }
static hipStream_t S(uintptr_t v) { return reinterpret_cast<hipStream_t>(v); }

static void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

PYBIND11_MODULE(_C, m) {
  m.doc() = "mercury_amd CDNA4 (gfx950) kernels";

  m.def("igemm", [](uintptr_t src, uintptr_t wt, uintptr_t out, int ldo, uintptr_t bias,
                    uintptr_t stats, int stats_ld, int group_rows, int accumulate, uintptr_t slab,
                    int SH, int SW, int SC, int RP, int RQ, int R, int Sk, int stride, int pad, int Kc,
                    int Ncols, int M, int bm, int bn, int splits, bool trans, uintptr_t st,
                    uintptr_t bw_out, uintptr_t bw_y, uintptr_t bw_stats, uintptr_t bw_y2,
                    uintptr_t bw_stats2, uintptr_t bw_sums, float bw_inv_count, float bw_eps,
                    int bw_act) {
    if (stats && bw_sums)   // the epilogue reduces both through one LDS scratch
      throw std::invalid_argument("igemm: forward BN stats and backward BN sums are exclusive");
    ConvGeom g{SH, SW, SC, RP, RQ, R, Sk, stride, pad, Kc, Ncols, M};
    EpiParams e{P<bf16>(out), ldo, P<const float>(bias), P<float>(stats), stats_ld, group_rows,
                accumulate, P<float>(slab), P<const bf16>(bw_out), P<const bf16>(bw_y),
                P<const float>(bw_stats), P<const bf16>(bw_y2), P<const float>(bw_stats2),
                P<float>(bw_sums), bw_inv_count, bw_eps, bw_act};
    igemm_launch(P<const bf16>(src), P<const bf16>(wt), g, e, bm, bn, splits, trans, S(st));
    check_launch("igemm");
  });
  // two independent forward convs (plain input, same tile) in one launch; each conv is
  // (src, wt, out, ldo, stats, stats_ld, group_rows, slab, SH, SW, SC, RP, RQ, R, S, stride, pad,
  //  Kc, Ncols, M, splits) as int64 values; returns 0 if there is no instantiation
  m.def("igemm_dual", [](std::vector<int64_t> a, std::vector<int64_t> b, int bm, int bn,
                         uintptr_t st) {
    if (a.size() != 21 || b.size() != 21) throw std::invalid_argument("igemm_dual: 21 values each");
    auto geo = [](const std::vector<int64_t>& v) {
      return ConvGeom{(int)v[8], (int)v[9], (int)v[10], (int)v[11], (int)v[12], (int)v[13],
                      (int)v[14], (int)v[15], (int)v[16], (int)v[17], (int)v[18], (int)v[19]};
    };
    auto epi = [](const std::vector<int64_t>& v) {
      return EpiParams{P<bf16>((uintptr_t)v[2]), (int)v[3], nullptr, P<float>((uintptr_t)v[4]),
                       (int)v[5], (int)v[6], 0, P<float>((uintptr_t)v[7]), nullptr, nullptr,
                       nullptr, nullptr, nullptr, nullptr, 0.f, 0.f, 0};
    };
    const int ok = igemm_dual_launch(P<const bf16>((uintptr_t)a[0]), P<const bf16>((uintptr_t)a[1]),
                                     geo(a), epi(a), (int)a[20], P<const bf16>((uintptr_t)b[0]),
                                     P<const bf16>((uintptr_t)b[1]), geo(b), epi(b), (int)b[20], bm,
                                     bn, S(st));
    if (ok) check_launch("igemm_dual");
    return ok;
  });
  // stride-2 dgrad by parity classes (one launch); returns 0 if the conv does not qualify
  m.def("dgrad_s2", [](uintptr_t dy, uintptr_t wt, uintptr_t dx, int ldo, int accumulate, int SH,
                       int SW, int SC, int R, int Sk, int stride, int pad, int Ncols, int bm,
                       int bn, int H, int W, int N, uintptr_t st, uintptr_t bw_out, uintptr_t bw_y,
                       uintptr_t bw_stats, uintptr_t bw_y2, uintptr_t bw_stats2, uintptr_t bw_sums,
                       float bw_inv_count, float bw_eps, int bw_act) {
    ConvGeom g{SH, SW, SC, H, W, R, Sk, stride, pad, R * Sk * SC / 8, Ncols, N * H * W};
    EpiParams e{P<bf16>(dx), ldo, nullptr, nullptr, 0, N * H * W, accumulate, nullptr,
                P<const bf16>(bw_out), P<const bf16>(bw_y), P<const float>(bw_stats),
                P<const bf16>(bw_y2), P<const float>(bw_stats2), P<float>(bw_sums), bw_inv_count,
                bw_eps, bw_act};
    const int ok = dgrad_s2_launch(P<const bf16>(dy), P<const bf16>(wt), g, e, bm, bn, H, W, N,
                                   S(st));
    if (ok) check_launch("dgrad_s2");
    return ok;
  });
  m.def("conv_bwd_pair_s2", [](uintptr_t dy, uintptr_t wt, uintptr_t dx, int ldo, int accumulate,
                               int SH, int SW, int SC, int R, int Sk, int stride, int pad,
                               int Ncols, int bm, int bn, int H, int W, int N, uintptr_t bw_out,
                               uintptr_t bw_y, uintptr_t bw_stats, uintptr_t bw_y2,
                               uintptr_t bw_stats2, uintptr_t bw_sums, float bw_inv_count,
                               float bw_eps, int bw_act, uintptr_t x, uintptr_t dw, int C, int Pp,
                               int Q, int K, int Creal, int wbm, int wbn, int wsplits,
                               uintptr_t wslab, uintptr_t st) {
    ConvGeom g{SH, SW, SC, H, W, R, Sk, stride, pad, R * Sk * SC / 8, Ncols, N * H * W};
    EpiParams e{P<bf16>(dx), ldo, nullptr, nullptr, 0, N * H * W, accumulate, nullptr,
                P<const bf16>(bw_out), P<const bf16>(bw_y), P<const float>(bw_stats),
                P<const bf16>(bw_y2), P<const float>(bw_stats2), P<float>(bw_sums), bw_inv_count,
                bw_eps, bw_act};
    WgradGeom wg{N, H, W, C, Pp, Q, K, R, Sk, stride, pad, Creal, nullptr, P<float>(wslab)};
    const int ok = conv_bwd_pair_s2_launch(P<const bf16>(dy), P<const bf16>(wt), g, e, bm, bn, H,
                                           W, N, P<const bf16>(x), wg, P<float>(dw), wbm, wbn,
                                           wsplits, S(st));
    if (ok) check_launch("conv_bwd_pair_s2");
    return ok;
  });
  m.attr("SUMS_R") = SUMS_R;   // replicas of the BN-backward sums ([SUMS_R][3][C])
  // 1x1 conv as a persistent LDS-DMA GEMM (pgemm.hip); returns 0 if unsupported
  m.def("pgemm", [](uintptr_t a, uintptr_t b, uintptr_t out, uintptr_t stats, int M, int N, int K,
                    int ldo, int stats_ld, int group_rows, long long a_bytes, long long b_bytes,
                    long long out_bytes, int H, int W, int Pp, int Q, int stride, int bn, int grid,
                    uintptr_t st, int p_mode, uintptr_t p_stats, uintptr_t p_rmean,
                    uintptr_t p_rvar, uintptr_t p_gamma, uintptr_t p_beta, float p_inv_count,
                    float p_eps, int p_act, int p_group_rows, int p_G, uintptr_t p_coef,
                    uintptr_t p_res, uintptr_t p_keep, long long p_res_bytes,
                    long long p_keep_bytes, long long p_coef_bytes) {
    const long long lim = 0xFFFFFF00LL;
    if (a_bytes >= lim || b_bytes >= lim || out_bytes >= lim || p_res_bytes >= lim ||
        p_keep_bytes >= lim || p_coef_bytes >= lim)
      throw std::invalid_argument("pgemm: tensors must be < 4 GB (32-bit buffer offsets)");
    PgemmArgs g{P<const bf16>(a), P<const bf16>(b), P<bf16>(out), P<float>(stats), M, N, K, ldo,
                stats_ld, group_rows, (unsigned)a_bytes, (unsigned)b_bytes, (unsigned)out_bytes,
                H, W, Pp, Q, stride};
    PgemmPro pr{p_mode, P<const float>(p_stats), P<const float>(p_rmean), P<const float>(p_rvar),
                P<const float>(p_gamma), P<const float>(p_beta), p_inv_count, p_eps, p_act,
                p_group_rows, p_G, P<float>(p_coef), P<const bf16>(p_res), P<bf16>(p_keep),
                (unsigned)p_res_bytes, (unsigned)p_keep_bytes, (unsigned)p_coef_bytes};
    // bn == 0: the panel-resident narrow-input kernel (pwconv.hip) instead
    const int ok = bn == 0 ? pwconv_launch(g, S(st), &pr) : pgemm_launch(g, bn, grid, S(st), &pr);
    check_launch(bn == 0 ? "pwconv" : "pgemm");
    return ok;
  });
  // forward conv whose A operand is BN-applied + activated on load (ProParams, igemm.h)
  m.def("igemm_pro", [](uintptr_t src, uintptr_t wt, uintptr_t out, int ldo, uintptr_t bias,
                        uintptr_t stats, int stats_ld, int group_rows, uintptr_t slab, int SH,
                        int SW, int SC, int RP, int RQ, int R, int Sk, int stride, int pad, int Kc,
                        int Ncols, int M, int bm, int bn, int splits, uintptr_t st,
                        uintptr_t p_stats, uintptr_t p_rmean, uintptr_t p_rvar, uintptr_t p_gamma,
                        uintptr_t p_beta, uintptr_t p_keep, int p_group_rows, float p_inv_count,
                        float p_eps, int p_act, int p_keep_tap, uintptr_t p_res) {
    ConvGeom g{SH, SW, SC, RP, RQ, R, Sk, stride, pad, Kc, Ncols, M};
    EpiParams e{P<bf16>(out), ldo, P<const float>(bias), P<float>(stats), stats_ld, group_rows, 0,
                P<float>(slab), nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0.f, 0.f, 0};
    ProParams pr{P<const float>(p_stats), P<const float>(p_rmean), P<const float>(p_rvar),
                 P<const float>(p_gamma), P<const float>(p_beta), P<bf16>(p_keep), p_group_rows,
                 p_inv_count, p_eps, p_act, p_keep_tap, P<const bf16>(p_res)};
    igemm_launch(P<const bf16>(src), P<const bf16>(wt), g, e, bm, bn, splits, false, S(st), &pr);
    check_launch("igemm_pro");
  });
  // halo-tile forward conv (hconv.hip) with the producer's BN (+ residual / shortcut BN) +
  // activation applied while staging its input
  m.def("hconv", [](uintptr_t src, uintptr_t wt, uintptr_t out, uintptr_t bias, uintptr_t stats,
                    int group_rows, uintptr_t slab, const std::vector<int>& geo, int bm, int bn,
                    int splits, uintptr_t st, int mode, uintptr_t p_stats, uintptr_t p_rmean,
                    uintptr_t p_rvar, uintptr_t p_gamma, uintptr_t p_beta, int p_group_imgs,
                    float p_inv_count, float p_eps, int p_act) {
    if (geo.size() != 21) throw std::invalid_argument("hconv: geometry needs 21 ints");
    if (geo[19] < 0 || geo[19] > 7) throw std::invalid_argument("hconv: SWA in 0..7");
    if (geo[20] < 0 || geo[20] > 4096) throw std::invalid_argument("hconv: PGRID in 0..4096");
    HconvGeom g{geo[0], geo[1], geo[2], geo[3], geo[4], geo[5], geo[6], geo[7], geo[8], geo[9],
                geo[10], geo[11], geo[12], geo[13], geo[14], geo[15], geo[16], geo[17], geo[18],
                geo[19], geo[20], 0, nullptr};
    const int K = geo[6];
    EpiParams e{P<bf16>(out), K, P<const float>(bias), P<float>(stats), K, group_rows, 0,
                P<float>(slab), nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0.f, 0.f, 0};
    HconvPro pr{mode, P<const float>(p_stats), P<const float>(p_rmean), P<const float>(p_rvar),
                P<const float>(p_gamma), P<const float>(p_beta), p_group_imgs, p_inv_count, p_eps,
                p_act};
    const int ok = hconv_launch(P<const bf16>(src), P<const bf16>(wt), g, e, pr, bm, bn, splits,
                                S(st));
    if (!ok) throw std::invalid_argument("hconv: tile not instantiated");
    check_launch("hconv");
  });
  m.def("conv_bwd_pair", [](uintptr_t dy, uintptr_t wt, uintptr_t dx, int ldo, int accumulate,
                            uintptr_t slab, int SH, int SW, int SC, int RP, int RQ, int R, int Sk,
                            int stride, int pad, int Kc, int Ncols, int M, int bm, int bn,
                            int splits, uintptr_t bw_out, uintptr_t bw_y, uintptr_t bw_stats,
                            uintptr_t bw_y2, uintptr_t bw_stats2, uintptr_t bw_sums,
                            float bw_inv_count, float bw_eps, int bw_act, uintptr_t x,
                            uintptr_t dw, int N, int H, int W, int C, int Pp, int Q, int K,
                            int Creal, int wbm, int wbn, int wsplits, uintptr_t wslab,
                            uintptr_t st) {
    ConvGeom g{SH, SW, SC, RP, RQ, R, Sk, stride, pad, Kc, Ncols, M};
    EpiParams e{P<bf16>(dx), ldo, nullptr, nullptr, 0, M, accumulate, P<float>(slab),
                P<const bf16>(bw_out), P<const bf16>(bw_y), P<const float>(bw_stats),
                P<const bf16>(bw_y2), P<const float>(bw_stats2), P<float>(bw_sums), bw_inv_count,
                bw_eps, bw_act};
    WgradGeom wg{N, H, W, C, Pp, Q, K, R, Sk, stride, pad, Creal, nullptr, P<float>(wslab)};
    const int ok = conv_bwd_pair_launch(P<const bf16>(dy), P<const bf16>(wt), g, e, bm, bn, splits,
                                        P<const bf16>(x), wg, P<float>(dw), wbm, wbn, wsplits, S(st));
    if (ok) check_launch("conv_bwd_pair");
    return ok;
  });
  // a block's last-conv pair (conv_bwd_pair's arguments, without the stream) and its shortcut's
  // stride-2 pair (conv_bwd_pair_s2's, 64 x 64 tiles) in one launch; returns 0 if unsupported
  m.def("conv_bwd_pair_sc", [](py::tuple a, py::tuple b, uintptr_t st) {
    if (a.size() != 44 || b.size() != 38) throw std::invalid_argument("conv_bwd_pair_sc: arity");
    auto U = [](const py::tuple& t, int i) { return t[i].cast<uintptr_t>(); };
    auto I = [](const py::tuple& t, int i) { return t[i].cast<int>(); };
    auto F = [](const py::tuple& t, int i) { return t[i].cast<float>(); };
    // A: dy wt dx ldo accumulate slab SH SW SC RP RQ R Sk stride pad Kc Ncols M bm bn splits
    //    bw_out bw_y bw_stats bw_y2 bw_stats2 bw_sums bw_inv_count bw_eps bw_act x dw N H W C Pp
    //    Q K Creal wbm wbn wsplits wslab
    ConvGeom gA{I(a, 6), I(a, 7), I(a, 8), I(a, 9), I(a, 10), I(a, 11), I(a, 12), I(a, 13),
                I(a, 14), I(a, 15), I(a, 16), I(a, 17)};
    EpiParams eA{P<bf16>(U(a, 2)), I(a, 3), nullptr, nullptr, 0, I(a, 17), I(a, 4),
                 P<float>(U(a, 5)), P<const bf16>(U(a, 21)), P<const bf16>(U(a, 22)),
                 P<const float>(U(a, 23)), P<const bf16>(U(a, 24)), P<const float>(U(a, 25)),
                 P<float>(U(a, 26)), F(a, 27), F(a, 28), I(a, 29)};
    WgradGeom wgA{I(a, 32), I(a, 33), I(a, 34), I(a, 35), I(a, 36), I(a, 37), I(a, 38), I(a, 11),
                  I(a, 12), I(a, 13), I(a, 14), I(a, 39), nullptr, P<float>(U(a, 43))};
    // B: dy wt dx ldo accumulate SH SW SC R Sk stride pad Ncols bm bn H W N bw_out bw_y bw_stats
    //    bw_y2 bw_stats2 bw_sums bw_inv_count bw_eps bw_act x dw C Pp Q K Creal wbm wbn wsplits
    //    wslab
    const int HB = I(b, 15), WB = I(b, 16), NB = I(b, 17);
    ConvGeom gB{I(b, 5), I(b, 6), I(b, 7), HB, WB, I(b, 8), I(b, 9), I(b, 10), I(b, 11),
                I(b, 8) * I(b, 9) * I(b, 7) / 8, I(b, 12), NB * HB * WB};
    EpiParams eB{P<bf16>(U(b, 2)), I(b, 3), nullptr, nullptr, 0, NB * HB * WB, I(b, 4), nullptr,
                 P<const bf16>(U(b, 18)), P<const bf16>(U(b, 19)), P<const float>(U(b, 20)),
                 P<const bf16>(U(b, 21)), P<const float>(U(b, 22)), P<float>(U(b, 23)), F(b, 24),
                 F(b, 25), I(b, 26)};
    WgradGeom wgB{NB, HB, WB, I(b, 29), I(b, 30), I(b, 31), I(b, 32), I(b, 8), I(b, 9), I(b, 10),
                  I(b, 11), I(b, 33), nullptr, P<float>(U(b, 37))};
    if (I(b, 13) != 64 || I(b, 14) != 64 || I(b, 34) != 64 || I(b, 35) != 64) return 0;
    const int ok = conv_bwd_pair_sc_launch(
        P<const bf16>(U(a, 0)), P<const bf16>(U(a, 1)), gA, eA, I(a, 18), I(a, 19), I(a, 20),
        P<const bf16>(U(a, 30)), wgA, P<float>(U(a, 31)), I(a, 40), I(a, 41), I(a, 42),
        P<const bf16>(U(b, 0)), P<const bf16>(U(b, 1)), gB, eB, HB, WB, NB,
        P<const bf16>(U(b, 27)), wgB, P<float>(U(b, 28)), I(b, 36), S(st));
    if (ok) check_launch("conv_bwd_pair_sc");
    return ok;
  });
  m.def("comm_unique_id", []() { return py::bytes(comm_unique_id()); });
  m.def("comm_init", [](py::bytes id, int rank, int nranks) {
    return comm_init(std::string(id), rank, nranks);
  });
  m.def("comm_destroy", &comm_destroy);
  m.def("comm_allreduce", &comm_allreduce);
  m.def("comm_allgather", &comm_allgather);
  m.def("comm_broadcast", &comm_broadcast);
  m.def("comm_ring_allreduce", [](uintptr_t c, uintptr_t buf, long long count, uintptr_t work,
                                  int avg, uintptr_t st) {
    comm_ring_allreduce(c, buf, count, work, avg, st);
    check_launch("comm_ring_allreduce");
  });
  // the exchange kernels address a buffer through a buffer resource: 32-bit byte offsets
  auto xgmi_range = [](long long n, int bf, const char* who) {
    if (n < 0 || n * (bf ? 2 : 4) >= (1LL << 31))
      throw std::invalid_argument(std::string(who) + ": exchange must be < 2 GiB (32-bit offsets)");
  };
  m.def("xgmi_pack", [xgmi_range](uintptr_t src, uintptr_t xbuf, long long n, int bf, uintptr_t st) {
    xgmi_range(n, bf, "xgmi_pack");
    xgmi_pack(P<const float>(src), P<void>(xbuf), n, bf, S(st));
    check_launch("xgmi_pack");
  });
  m.def("xgmi_reduce_scatter", [xgmi_range](const std::vector<uintptr_t>& peers, int rank,
                                            long long n, int bf, float scale, uintptr_t st) {
    xgmi_range(n, bf, "xgmi_reduce_scatter");
    if (peers.empty() || (int)peers.size() > xgmi_max_ranks() || n % 4)
      throw std::invalid_argument("xgmi_reduce_scatter: 1..8 peers, n % 4 == 0");
    std::vector<const void*> p(peers.size());
    for (size_t i = 0; i < peers.size(); ++i) p[i] = P<const void>(peers[i]);
    xgmi_reduce_scatter(p.data(), (int)p.size(), rank, n, bf, scale, S(st));
    check_launch("xgmi_reduce_scatter");
  });
  m.def("xgmi_all_gather", [xgmi_range](const std::vector<uintptr_t>& peers, long long n, int bf,
                                        uintptr_t dst, uintptr_t st) {
    xgmi_range(n, bf, "xgmi_all_gather");
    if (peers.empty() || (int)peers.size() > xgmi_max_ranks() || n % 4)
      throw std::invalid_argument("xgmi_all_gather: 1..8 peers, n % 4 == 0");
    std::vector<const void*> p(peers.size());
    for (size_t i = 0; i < peers.size(); ++i) p[i] = P<const void>(peers[i]);
    xgmi_all_gather(p.data(), (int)p.size(), n, bf, P<float>(dst), S(st));
    check_launch("xgmi_all_gather");
  });
  m.def("xgmi_barrier", [](const std::vector<uintptr_t>& flag_areas, int rank, uintptr_t epoch,
                           double timeout_s, uintptr_t err, uintptr_t st) {
    if (flag_areas.empty() || (int)flag_areas.size() > xgmi_max_ranks() || rank < 0 ||
        rank >= (int)flag_areas.size())
      throw std::invalid_argument("xgmi_barrier: 1..8 flag areas, 0 <= rank < W");
    std::vector<const void*> p(flag_areas.size());
    for (size_t i = 0; i < flag_areas.size(); ++i) p[i] = P<const void>(flag_areas[i]);
    xgmi_barrier(p.data(), (int)p.size(), rank, P<unsigned>(epoch), timeout_s, P<int>(err), S(st));
    check_launch("xgmi_barrier");
  });
  m.def("xgmi_flag_bytes", &xgmi_flag_bytes);
  m.def("xgmi_ipc_handle", [](uintptr_t p) { return py::bytes(xgmi_ipc_handle(p)); });
  m.def("xgmi_ipc_open", [](py::bytes h) { return xgmi_ipc_open(std::string(h)); });
  m.def("xgmi_ipc_close", &xgmi_ipc_close);
  m.def("xgmi_malloc", &xgmi_malloc);
  m.def("xgmi_free", &xgmi_free);
  m.def("add_f32", [](uintptr_t dst, uintptr_t src, long long n, uintptr_t st) {
    add_f32(P<float>(dst), P<const float>(src), n, S(st));
    check_launch("add_f32");
  });
  // stream-order race detector (runtime.hip)
  m.def("order_check", [](uintptr_t o, int slot, int ref, int mult, int add, int ge, int tick,
                          int at, uintptr_t st) {
    order_check_launch(P<int>(o), slot, ref, mult, add, ge, tick, at, S(st));
    check_launch("order_check");
  });
  // one-graph DP train replay (EngineOptions.comm_events): the train segments' captured graphs
  // chained as child-graph nodes with an event-record NODE after each bucket's segment, in ONE
  // linear executable graph.  hipGraphLaunch enqueues the record nodes in order, so a
  // hipStreamWaitEvent issued after the launch waits on that node of this replay.  (torch's
  // ROCm build refuses torch.cuda.Event(external=True) and HIP refuses hipEventRecordExternal
  // inside a capture, so the nodes are added explicitly.)
  m.def("ext_event_create", []() {
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
      throw std::runtime_error("hipEventCreateWithFlags failed");
    return reinterpret_cast<uintptr_t>(e);
  });
  m.def("ext_event_wait", [](uintptr_t st, uintptr_t e) {
    const hipError_t r = hipStreamWaitEvent(S(st), reinterpret_cast<hipEvent_t>(e), 0);
    if (r != hipSuccess)
      throw std::runtime_error(std::string("hipStreamWaitEvent: ") + hipGetErrorString(r));
  });
  m.def("ext_event_destroy", [](uintptr_t e) { (void)hipEventDestroy(reinterpret_cast<hipEvent_t>(e)); });
  m.def("graph_chain", [](std::vector<uintptr_t> graphs, std::vector<uintptr_t> events) {
    if (graphs.size() != events.size()) throw std::runtime_error("graph_chain: one event slot per graph");
    auto ck = [](hipError_t r, const char* what) {
      if (r != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(r));
    };
    hipGraph_t parent = nullptr;
    ck(hipGraphCreate(&parent, 0), "hipGraphCreate");
    hipGraphNode_t prev = nullptr;
    for (size_t k = 0; k < graphs.size(); ++k) {
      hipGraphNode_t n = nullptr;
      ck(hipGraphAddChildGraphNode(&n, parent, prev ? &prev : nullptr, prev ? 1 : 0,
                                   reinterpret_cast<hipGraph_t>(graphs[k])),
         "hipGraphAddChildGraphNode");
      prev = n;
      if (events[k]) {
        ck(hipGraphAddEventRecordNode(&n, parent, &prev, 1, reinterpret_cast<hipEvent_t>(events[k])),
           "hipGraphAddEventRecordNode");
        prev = n;
      }
    }
    hipGraphExec_t ex = nullptr;
    ck(hipGraphInstantiate(&ex, parent, nullptr, nullptr, 0), "hipGraphInstantiate");
    ck(hipGraphDestroy(parent), "hipGraphDestroy");
    return reinterpret_cast<uintptr_t>(ex);
  });
  m.def("graph_launch", [](uintptr_t ex, uintptr_t st) {
    const hipError_t r = hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(ex), S(st));
    if (r != hipSuccess) throw std::runtime_error(std::string("hipGraphLaunch: ") + hipGetErrorString(r));
  });
  m.def("graph_exec_destroy", [](uintptr_t ex) {
    (void)hipGraphExecDestroy(reinterpret_cast<hipGraphExec_t>(ex));
  });
  m.def("igemm_stamps", [](int n) {   // diagnostic build only (MERCURY_STAMPS); else empty
    std::vector<unsigned long long> v((size_t)n * 12, 0ull);
    if (!igemm_read_stamps(v.data(), n)) v.clear();
    return v;
  });
  m.def("hconv_configure", &hconv_configure);
// persistent halo grid (0: half the CUs), waves
  m.def("hconv_stamps", [](int n) {   // diagnostic build only (MERCURY_STAMPS); else empty
    std::vector<unsigned long long> v((size_t)n * 12, 0ull);
    if (!hconv_read_stamps(v.data(), n)) v.clear();
    return v;
  });
  m.def("igemm_slab_bytes", [](int M, int Ncols, int bm, int bn, int splits) {
    ConvGeom g{};
    g.M = M;
    g.Ncols = Ncols;
    return igemm_slab_bytes(g, bm, bn, splits);
  });

  m.def("wgrad", [](uintptr_t dy, uintptr_t x, uintptr_t dw, int N, int H, int W, int C, int Pp,
                    int Q, int K, int R, int Sk, int stride, int pad, int Creal, int bm, int bn,
                    int splits, uintptr_t slab, uintptr_t st) {
    WgradGeom g{N, H, W, C, Pp, Q, K, R, Sk, stride, pad, Creal, nullptr, P<float>(slab)};
    wgrad_launch(P<const bf16>(dy), P<const bf16>(x), g, P<float>(dw), bm, bn, splits, S(st));
    check_launch("wgrad");
  });

  m.def("bn_configure", &bn_configure);
  m.def("bn_apply", [](uintptr_t y, uintptr_t stats, uintptr_t gamma, uintptr_t beta,
                       uintptr_t rmean, uintptr_t rvar, int use_running, int res_mode, uintptr_t res,
                       uintptr_t stats2, uintptr_t gamma2, uintptr_t beta2, uintptr_t rmean2,
                       uintptr_t rvar2, uintptr_t out, int M, int C, int group_rows, int act,
                       float eps, uintptr_t st) {
    BnApplyArgs a{P<const bf16>(y), P<const float>(stats), P<const float>(gamma),
                  P<const float>(beta), P<const float>(rmean), P<const float>(rvar), use_running,
                  res_mode, P<const bf16>(res), P<const float>(stats2), P<const float>(gamma2),
                  P<const float>(beta2), P<const float>(rmean2), P<const float>(rvar2),
                  P<bf16>(out), M, C, group_rows, act, eps};
    bn_apply_launch(a, S(st));
    check_launch("bn_apply");
  });

  m.def("bn_bwd", [](uintptr_t dout, uintptr_t out, uintptr_t y, uintptr_t stats, uintptr_t gamma,
                     uintptr_t y2, uintptr_t stats2, uintptr_t gamma2, uintptr_t sums, uintptr_t dy,
                     uintptr_t dy2, uintptr_t dz, uintptr_t dgamma, uintptr_t dbeta,
                     uintptr_t dgamma2, uintptr_t dbeta2, int M, int C, int act, float eps,
                     uintptr_t st, int phases) {
    BnBwdArgs a{P<const bf16>(dout), P<const bf16>(out), P<const bf16>(y), P<const float>(stats),
                P<const float>(gamma), P<const bf16>(y2), P<const float>(stats2),
                P<const float>(gamma2), P<float>(sums), P<bf16>(dy), P<bf16>(dy2), P<bf16>(dz),
                P<float>(dgamma), P<float>(dbeta), P<float>(dgamma2), P<float>(dbeta2), M, C, act,
                eps, phases};
    bn_bwd_launch(a, S(st));
    check_launch("bn_bwd");
  });

  m.def("pack_bn_table", [](const std::vector<std::vector<double>>& rows) {
    std::vector<BnRunEntry> v;
    for (const auto& r : rows) {
      BnRunEntry e{};
      e.rmean = P<float>((uintptr_t)r[0]);
      e.rvar = P<float>((uintptr_t)r[1]);
      e.stats_train = P<const float>((uintptr_t)r[2]);
      e.stats_score = P<const float>((uintptr_t)r[3]);
      e.nbt = P<long long>((uintptr_t)r[4]);
      e.C = (int)r[5];
      e.n_train = (int)r[6];
      e.n_score = (int)r[7];
      e.cnt_train = (float)r[8];
      e.cnt_score = (float)r[9];
      v.push_back(e);
    }
    return py::bytes(reinterpret_cast<const char*>(v.data()), v.size() * sizeof(BnRunEntry));
  });
  m.def("bn_running", [](uintptr_t tab, int nlayers, int maxC, float momentum, uintptr_t st) {
    bn_running_launch(P<const BnRunEntry>(tab), nlayers, maxC, momentum, S(st));
    check_launch("bn_running");
  });

  m.def("head_fwd", [](uintptr_t act, uintptr_t w, uintptr_t b, uintptr_t label, uintptr_t isw,
                       uintptr_t pooled, uintptr_t logits, uintptr_t dlogits, uintptr_t losses,
                       uintptr_t meters, int B, int HW, int C, int classes, int mode, uintptr_t st,
                       int score_kind, uintptr_t bn_res, uintptr_t bn_stats, uintptr_t bn_rmean,
                       uintptr_t bn_rvar, uintptr_t bn_gamma, uintptr_t bn_beta,
                       float bn_inv_count, float bn_eps, int bn_group_imgs, int bn_act) {
    HeadArgs a{P<const bf16>(act), P<const float>(w), P<const float>(b), P<const int>(label),
               P<const float>(isw), P<float>(pooled), P<float>(logits), P<float>(dlogits),
               P<float>(losses), P<float>(meters), B, HW, C, classes, mode, 0, score_kind, 0};
    if (bn_gamma) {
      if (!pooled || C % 8 || bn_group_imgs <= 0 || (!bn_stats && !(bn_rmean && bn_rvar)))
        throw std::invalid_argument("head_fwd: BN prologue needs pooled, C % 8 == 0, stats");
      a.bn_res = P<const bf16>(bn_res);
      a.bn_stats = P<const float>(bn_stats);
      a.bn_rmean = P<const float>(bn_rmean);
      a.bn_rvar = P<const float>(bn_rvar);
      a.bn_gamma = P<const float>(bn_gamma);
      a.bn_beta = P<const float>(bn_beta);
      a.bn_inv_count = bn_inv_count;
      a.bn_eps = bn_eps;
      a.bn_group_imgs = bn_group_imgs;
      a.bn_act = bn_act;
    }
    head_fwd_launch(a, S(st));
    check_launch("head_fwd");
  });
  // speech-VGG head (flatten -> fc1 -> fc2 -> log-softmax CE), head.hip
  m.def("mlp_head_fwd", [](uintptr_t x, uintptr_t w1, uintptr_t b1, uintptr_t w2, uintptr_t b2,
                           uintptr_t h1, uintptr_t logits, uintptr_t label, uintptr_t isw,
                           uintptr_t dlogits, uintptr_t losses, uintptr_t meters, int B, int F,
                           int H1, int K, int mode, int score_kind, int splits, uintptr_t st) {
    mlp_head_fwd_launch(P<const bf16>(x), P<const bf16>(w1), P<const float>(b1),
                        P<const float>(w2), P<const float>(b2), P<float>(h1), P<float>(logits), B,
                        F, H1, K, splits, S(st));
    HeadArgs a{nullptr, P<const float>(w2), P<const float>(b2), P<const int>(label),
               P<const float>(isw), P<float>(h1), P<float>(logits), P<float>(dlogits),
               P<float>(losses), P<float>(meters), B, 1, H1, K, mode, 0, score_kind, 1};
    head_loss_launch(a, S(st));
    check_launch("mlp_head_fwd");
  });
  m.def("mlp_head_bwd", [](uintptr_t dlogits, uintptr_t h1, uintptr_t x, uintptr_t w1, uintptr_t w2,
                           uintptr_t dh1, uintptr_t dw1, uintptr_t db1, uintptr_t dw2, uintptr_t db2,
                           uintptr_t dx, int B, int F, int H1, int K, uintptr_t st) {
    mlp_head_bwd_launch(P<const float>(dlogits), P<const float>(h1), P<const bf16>(x),
                        P<const bf16>(w1), P<const float>(w2), P<float>(dh1), P<float>(dw1),
                        P<float>(db1), P<float>(dw2), P<float>(db2), P<bf16>(dx), B, F, H1, K, S(st));
    check_launch("mlp_head_bwd");
  });
  m.def("head_bwd", [](uintptr_t pooled, uintptr_t dlogits, uintptr_t w, uintptr_t dw, uintptr_t db,
                       uintptr_t dact, int B, int HW, int C, int classes, uintptr_t st,
                       uintptr_t bw_out, uintptr_t bw_y, uintptr_t bw_stats, uintptr_t bw_y2,
                       uintptr_t bw_stats2, uintptr_t bw_sums, float bw_inv_count, float bw_eps,
                       int bw_act) {
    HeadBwdArgs a{P<const float>(pooled), P<const float>(dlogits), P<const float>(w), P<float>(dw),
                  P<float>(db), P<bf16>(dact), B, HW, C, classes, P<const bf16>(bw_out),
                  P<const bf16>(bw_y), P<const float>(bw_stats), P<const bf16>(bw_y2),
                  P<const float>(bw_stats2), P<float>(bw_sums), bw_inv_count, bw_eps, bw_act};
    const int ok = head_bwd_launch(a, S(st));
    check_launch("head_bwd");
    return ok;
  });

  m.def("pool_build", [](uintptr_t shard, uintptr_t labels, uintptr_t ctrl, uintptr_t pool,
                         uintptr_t pool_label, uintptr_t pool_index, int Ns, int H, int W, int Pn,
                         int batch, int pad, int flip, int augment, int shuffle, uint32_t seed,
                         std::vector<float> mean, std::vector<float> inv_std, uintptr_t st,
                         int prebuilt, uintptr_t zero, int nzero) {
    PoolBuildArgs a{P<const uint8_t>(shard), P<const int64_t>(labels), P<const int64_t>(ctrl),
                    P<bf16>(pool), P<int>(pool_label), P<int>(pool_index), Ns, H, W, Pn, batch,
                    pad, flip, augment, shuffle, seed, {mean[0], mean[1], mean[2]},
                    {inv_std[0], inv_std[1], inv_std[2]}, prebuilt, P<float>(zero), nzero};
    pool_build_launch(a, S(st));
    check_launch("pool_build");
  });
  m.def("is_sample", [](uintptr_t losses, uintptr_t ema, uintptr_t ctrl, uintptr_t idx, uintptr_t w,
                        uintptr_t meters, int Pn, int B, int group, int importance, float alpha,
                        float ema_alpha, uint32_t seed, uintptr_t st, int alias, uintptr_t gl,
                        int W) {
    if (group <= 0 || Pn % group || Pn / group > 1024)
      throw std::runtime_error("is_sample: pool must be 1..1024 groups of `group` samples");
    if (alias && is_sample_lds(Pn, 1) > 128 * 1024) alias = 0;   // table beyond LDS: inverse CDF
    IsSampleArgs a{P<const float>(losses), P<float>(ema), P<int64_t>(ctrl), P<int>(idx), P<float>(w),
                   P<float>(meters), Pn, B, group, importance, alpha, ema_alpha, seed, alias,
                   P<const float>(gl), W};
    is_sample_launch(a, S(st));
    check_launch("is_sample");
  });
  m.def("gather", [](uintptr_t pool, uintptr_t pool_label, uintptr_t pool_index, uintptr_t idx,
                     uintptr_t batch, uintptr_t batch_label, uintptr_t batch_index, int B,
                     int chunks_per_img, uintptr_t st) {
    GatherArgs a{P<const bf16>(pool), P<const int>(pool_label), P<const int>(pool_index),
                 P<const int>(idx), P<bf16>(batch), P<int>(batch_label), P<int>(batch_index), B,
                 chunks_per_img};
    gather_launch(a, S(st));
    check_launch("gather");
  });
  m.def("table_num_segments", &table_num_segments);
  m.def("table_scalars_bytes", []() { return (int)sizeof(TableScalars); });
  m.def("table_scatter", [](uintptr_t imp, uintptr_t grp, uintptr_t losses, uintptr_t index,
                            uintptr_t stamp, int start, int n, int N, int gi, uintptr_t st) {
    TableScatterArgs a{P<float>(imp), P<int>(grp), P<const float>(losses), P<const int>(index),
                       P<const int64_t>(stamp), start, n, N, gi};
    table_scatter_launch(a, S(st));
    check_launch("table_scatter");
  });
  m.def("table_sample", [](uintptr_t imp, uintptr_t grp, int N, int gi, uintptr_t gi_dev,
                           uintptr_t part, uintptr_t prefix, uintptr_t sc, uintptr_t counter,
                           int ndraw, uint32_t seed, uintptr_t out, uintptr_t out32, uintptr_t st) {
    TableSampleArgs a{P<const float>(imp), P<const int>(grp), N, gi, P<const int64_t>(gi_dev),
                      P<float2>(part), P<double>(prefix), P<TableScalars>(sc), P<int64_t>(counter),
                      ndraw, seed, P<int64_t>(out), P<int>(out32)};
    table_sample_launch(a, S(st));
    check_launch("table_sample");
  });
  m.def("table_weights", [](uintptr_t pos, int ndraw, uintptr_t imp, uintptr_t sc,
                            uintptr_t pool_index, int Ns, int npool, uintptr_t idx, uintptr_t isw,
                            uintptr_t meters, uintptr_t st) {
    table_weights_launch(P<const int>(pos), ndraw, P<const float>(imp), (const void*)sc,
                         P<const int>(pool_index), Ns, npool, P<int>(idx), P<float>(isw),
                         P<float>(meters), S(st));
    check_launch("table_weights");
  });

  m.def("pack_opt_segs", [](const std::vector<std::vector<long long>>& rows) {
    std::vector<OptSeg> v;
    for (const auto& r : rows) {
      OptSeg s{};
      s.off = r[0];
      s.numel = (int)r[1];
      s.kind = (int)r[2];
      s.K = (int)r[3];
      s.R = (int)r[4];
      s.S = (int)r[5];
      s.C = (int)r[6];
      s.Cpad = (int)r[7];
      s.w_krsc = P<bf16>((uintptr_t)r[8]);
      s.w_crsk = P<bf16>((uintptr_t)r[9]);
      v.push_back(s);
    }
    return py::bytes(reinterpret_cast<const char*>(v.data()), v.size() * sizeof(OptSeg));
  });
  m.def("optimizer", [](uintptr_t p, uintptr_t g, uintptr_t mm, uintptr_t v, uintptr_t segs,
                        int nsegs, long long total, uintptr_t hyper, uintptr_t step, int algo,
                        int zero_grad, uintptr_t st, long long start) {
    OptArgs a{P<float>(p), P<float>(g), P<float>(mm), P<float>(v), P<const OptSeg>(segs), nsegs,
              total, P<const float>(hyper), P<const int64_t>(step), algo, zero_grad, start};
    optimizer_launch(a, S(st));
    check_launch("optimizer");
  });
  m.def("optimizer_fused", [](uintptr_t p, uintptr_t g, uintptr_t mm, uintptr_t v, uintptr_t segs,
                              int nsegs, long long total, uintptr_t hyper, uintptr_t step,
                              int algo, int zero_grad, uintptr_t jobs, int njobs, uintptr_t ew,
                              uintptr_t ewp, int new_, long long ew4, uintptr_t st) {
    OptArgs a{P<float>(p), P<float>(g), P<float>(mm), P<float>(v), P<const OptSeg>(segs), nsegs,
              total, P<const float>(hyper), P<const int64_t>(step), algo, zero_grad, 0};
    optimizer_fused_launch(a, P<const int>(jobs), njobs, P<const long long>(ew),
                           P<const long long>(ewp), new_, ew4, S(st));
    check_launch("optimizer_fused");
  });
  m.def("pack_weights", [](uintptr_t p, uintptr_t segs, int nsegs, long long total, uintptr_t st) {
    pack_weights_launch(P<const float>(p), P<const OptSeg>(segs), nsegs, total, S(st));
    check_launch("pack_weights");
  });
  m.def("transpose_weights", [](uintptr_t segs, uintptr_t jobs, int njobs, uintptr_t st) {
    transpose_weights_launch(P<const OptSeg>(segs), P<const int>(jobs), njobs, S(st));
    check_launch("transpose_weights");
  });
  m.def("step_begin", [](uintptr_t ctrl, uintptr_t st, uintptr_t z0, int n0, uintptr_t z1,
                         int n1) {
    step_begin_launch(P<int64_t>(ctrl), P<float>(z0), n0, P<float>(z1), n1, S(st));
    check_launch("step_begin");
  });

  m.def("quantize", [](uintptr_t x, uintptr_t out, uintptr_t ws, long long n, uint32_t seed,
                       uint64_t counter, uintptr_t st) {
    quantize_launch(P<const float>(x), P<float>(out), P<float>(ws), n, seed, counter, S(st));
    check_launch("quantize");
  });
  m.def("tern_pack", [](uintptr_t x, long long n, uintptr_t ws, uint32_t seed, uint64_t counter,
                        uintptr_t words, uintptr_t st, uintptr_t dctr) {
    tern_pack_launch(P<const float>(x), n, P<float>(ws), seed, counter, P<const long long>(dctr),
                     P<uint32_t>(words), S(st));
    check_launch("tern_pack");
  });
  m.def("tern_unpack", [](uintptr_t msgs, int W, long long n, float scale, uintptr_t out,
                          uintptr_t st) {
    tern_unpack_launch(P<const uint32_t>(msgs), W, n, scale, P<float>(out), S(st));
    check_launch("tern_unpack");
  });
  m.def("pool2d_fwd", [](uintptr_t x, uintptr_t y, uintptr_t argmax, int N, int H, int W, int C,
                         int Pp, int Q, int k, int stride, int pad, int is_max, uintptr_t st,
                         uintptr_t stats, uintptr_t gamma, uintptr_t beta, uintptr_t rmean,
                         uintptr_t rvar, int group_imgs, int act, float eps) {
    PoolArgs a{P<const bf16>(x), P<bf16>(y), P<uint8_t>(argmax), N, H, W, C, Pp, Q, k, stride,
               pad, is_max, P<const float>(stats), P<const float>(gamma), P<const float>(beta),
               P<const float>(rmean), P<const float>(rvar), group_imgs, act, eps};
    pool2d_fwd_launch(a, S(st));
    check_launch("pool2d_fwd");
  });
  m.def("maxpool2d_bwd", [](uintptr_t dy, uintptr_t argmax, uintptr_t dx, int N, int H, int W, int C,
                            int Pp, int Q, int k, int stride, int pad, uintptr_t st) {
    PoolArgs a{nullptr, nullptr, P<uint8_t>(argmax), N, H, W, C, Pp, Q, k, stride, pad, 1,
               nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, 0.f};
    maxpool2d_bwd_launch(a, P<const bf16>(dy), P<bf16>(dx), S(st));
    check_launch("maxpool2d_bwd");
  });
  m.def("dwconv_fwd", [](uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t stats, int N, int H, int W,
                         int C, int Pp, int Q, int stride, int pad, int group_rows, uintptr_t st,
                         uintptr_t p_stats, uintptr_t p_rmean, uintptr_t p_rvar, uintptr_t p_gamma,
                         uintptr_t p_beta, uintptr_t keep, float p_inv_count, float p_eps,
                         int p_act, int p_group_imgs) {
    if (p_gamma && (pad != 1 || (stride != 1 && stride != 2) || H != Pp * stride || W != Q * stride))
      throw std::invalid_argument("dwconv_fwd: input prologue needs a pad-1 'same' 3x3 conv");
    DwArgs a{P<const bf16>(x), P<const float>(w), P<bf16>(y), P<float>(stats), N, H, W, C, Pp, Q,
             stride, pad, group_rows, P<const float>(p_stats), P<const float>(p_rmean),
             P<const float>(p_rvar), P<const float>(p_gamma), P<const float>(p_beta), P<bf16>(keep),
             p_inv_count, p_eps, p_act, p_group_imgs > 0 ? p_group_imgs : N};
    dwconv_fwd_launch(a, S(st));
    check_launch("dwconv_fwd");
  });
  // stem conv (<= 4 input channels, taps x channels packed into k); returns 0 if unsupported
  m.def("stem_fwd", [](uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, uintptr_t stats,
                       int N, int H, int W, int K, int R, int stride, int pad, int Pp, int Q,
                       int group_imgs, uintptr_t st) {
    StemArgs a{P<const bf16>(x), P<const bf16>(w), P<const float>(bias), P<bf16>(y), P<float>(stats),
               N, H, W, K, R, stride, pad, Pp, Q, group_imgs, 0, 0};
    const int ok = stem_fwd_launch(a, S(st));
    check_launch("stem_fwd");
    return ok;
  });
  m.def("dwconv_wgrad_slab_floats", [](int N, int Pp, int Q, int C) {
    return (long long)dwconv_wgrad_slab_floats(N, Pp, Q, C);
  });
  m.def("dwconv_dgrad", [](uintptr_t dy, uintptr_t w, uintptr_t dx, int N, int H, int W, int C,
                           int Pp, int Q, int stride, int pad, uintptr_t st, uintptr_t bw_out,
                           uintptr_t bw_y, uintptr_t bw_stats, uintptr_t bw_sums,
                           float bw_inv_count, float bw_eps, int bw_act) {
    const DwBw bw{P<const bf16>(bw_out), P<const bf16>(bw_y), P<const float>(bw_stats),
                  P<float>(bw_sums), bw_inv_count, bw_eps, bw_act};
    dwconv_dgrad_launch(P<const bf16>(dy), P<const float>(w), P<bf16>(dx), N, H, W, C, Pp, Q, stride,
                        pad, S(st), bw_sums ? &bw : nullptr);
    check_launch("dwconv_dgrad");
  });
  m.def("dwconv_wgrad_blocks", &dwconv_wgrad_blocks);
  m.def("dwconv_bwd", [](uintptr_t dy, uintptr_t x, uintptr_t w, uintptr_t dx, uintptr_t dw, int N,
                         int H, int W, int C, int Pp, int Q, int stride, int pad, uintptr_t slab,
                         int reduce, uintptr_t st, uintptr_t bw_out, uintptr_t bw_y,
                         uintptr_t bw_stats, uintptr_t bw_sums, float bw_inv_count, float bw_eps,
                         int bw_act) {
    DwBw bw{P<const bf16>(bw_out), P<const bf16>(bw_y), P<const float>(bw_stats), P<float>(bw_sums),
            bw_inv_count, bw_eps, bw_act};
    dwconv_bwd_launch(P<const bf16>(dy), P<const bf16>(x), P<const float>(w), P<bf16>(dx),
                      P<float>(dw), N, H, W, C, Pp, Q, stride, pad, P<float>(slab),
                      bw_sums ? &bw : nullptr, reduce != 0, S(st));
    check_launch("dwconv_bwd");
  });
  m.def("dwconv_wgrad_reduce_batch", [](std::vector<uintptr_t> slabs, std::vector<uintptr_t> dws,
                                        std::vector<int> Cs, std::vector<int> nblks, uintptr_t st) {
    const size_t n = slabs.size();
    if (dws.size() != n || Cs.size() != n || nblks.size() != n)
      throw std::invalid_argument("dwconv_wgrad_reduce_batch: list lengths differ");
    std::vector<const float*> sp(n);
    std::vector<float*> dp(n);
    for (size_t i = 0; i < n; ++i) {
      sp[i] = P<const float>(slabs[i]);
      dp[i] = P<float>(dws[i]);
    }
    dwconv_wgrad_reduce_batch_launch(sp.data(), dp.data(), Cs.data(), nblks.data(), (int)n, S(st));
    check_launch("dwconv_wgrad_reduce_batch");
  });
  m.def("dwconv_wgrad", [](uintptr_t dy, uintptr_t x, uintptr_t dw, int N, int H, int W, int C,
                           int Pp, int Q, int stride, int pad, uintptr_t st, uintptr_t slab,
                           long long slab_floats) {
    dwconv_wgrad_launch(P<const bf16>(dy), P<const bf16>(x), P<float>(dw), N, H, W, C, Pp, Q, stride,
                        pad, S(st), P<float>(slab), (size_t)slab_floats);
    check_launch("dwconv_wgrad");
  });
  m.def("nchw_to_nhwc8", [](uintptr_t x, uintptr_t y, int N, int C, int H, int W, int Cpad,
                            uintptr_t st) {
    nchw_to_nhwc8_launch(P<const float>(x), P<bf16>(y), N, C, H, W, Cpad, S(st));
    check_launch("nchw_to_nhwc8");
  });
  m.def("arch", []() { return std::string("gfx950"); });
}
