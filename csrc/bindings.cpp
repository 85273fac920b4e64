// pybind11 bindings of the gfx950 kernels. Deliberately torch-ABI-free: Python passes raw
// device pointers (tensor.data_ptr()), sizes and the current HIP stream handle, so the
// extension only depends on the HIP runtime that torch itself loaded.
#include <pybind11/pybind11.h>
#include <hip/hip_runtime.h>
#include <pybind11/stl.h>
#include <cstdlib>
#include <string>
#include <vector>
#include "kernels.h"

namespace py = pybind11;
using uptr = uintptr_t;

#define P(x) reinterpret_cast<void*>(x)
#define CP(x) reinterpret_cast<const void*>(x)
#define FP(x) reinterpret_cast<float*>(x)
#define CFP(x) reinterpret_cast<const float*>(x)
#define ST(x) reinterpret_cast<hipStream_t>(x)

// DV_SYNC_CHECK=1 (or set_sync_check(True)): synchronise after every native launch so an
// asynchronous fault is reported by the op that caused it (the HIP_LAUNCH_BLOCKING /
// AMD_SERIALIZE_KERNEL debugging idiom, per op and without serialising other libraries).
static bool g_sync_check = [] {
  const char* v = std::getenv("DV_SYNC_CHECK");
  return v && v[0] && v[0] != '0';
}();

static void check_last(const char* what) {
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && g_sync_check) {
    e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipGetLastError();
  }
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

PYBIND11_MODULE(_C, m) {
  m.doc() = "deep_vision_amd native gfx950 kernels";
  m.attr("STAT_SHARDS") = DV_STAT_SHARDS;

  m.def("conv_fwd", [](uptr x, uptr w, uptr y, uptr bias, uptr stats, int Nb, int H, int W, int Cg, int ldx, int G,
                       int Kout, int P_, int Q, int R, int S, int sh, int sw, int ph, int pw, int dh, int dw, int tgather,
                       int OH, int OW, int osh, int osw, int oph, int opw, int ldy, int act, float slope, uptr res,
                       uptr st, uptr bnx, uptr bnbits, uptr bnprm, uptr bnacc, int bnmode, int bnact, float bnslope,
                       uptr resbits, int resact, float resslope, int reflect, int ksplit, uptr ypart, int zfill,
                       uptr bnx2, uptr bnprm2, uptr bnacc2, int w_ld, int w_kr, int w_ks) {
    ConvFwdArgs a{CP(x), CP(w), P(y), CFP(bias), FP(stats), Nb, H, W, Cg, ldx, G, Kout, P_, Q, R, S, sh, sw, ph, pw,
                  dh, dw, tgather, OH, OW, osh, osw, oph, opw, ldy, act, slope, CP(res),
                  CP(bnx), CP(bnbits), CFP(bnprm), FP(bnacc), bnmode, bnact, bnslope, CP(resbits), resact, resslope,
                  reflect, ksplit, FP(ypart), zfill, CP(bnx2), CFP(bnprm2), FP(bnacc2)};
    a.w_ld = w_ld; a.w_kr = w_kr; a.w_ks = w_ks;
    int r = dv_conv_fwd(a, ST(st));
    if (r < 0) throw std::runtime_error("conv_fwd: unsupported geometry (channels must be a multiple of 8)");
    check_last("conv_fwd");
    return r;
  }, py::arg("x"), py::arg("w"), py::arg("y"), py::arg("bias"), py::arg("stats"), py::arg("Nb"), py::arg("H"),
     py::arg("W"), py::arg("Cg"), py::arg("ldx"), py::arg("G"), py::arg("Kout"), py::arg("P"), py::arg("Q"), py::arg("R"),
     py::arg("S"), py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("dh"), py::arg("dw"),
     py::arg("tgather"), py::arg("OH"), py::arg("OW"), py::arg("osh"), py::arg("osw"), py::arg("oph"), py::arg("opw"),
     py::arg("ldy"), py::arg("act"), py::arg("slope"), py::arg("res"), py::arg("st"), py::arg("bnx") = 0,
     py::arg("bnbits") = 0, py::arg("bnprm") = 0, py::arg("bnacc") = 0, py::arg("bnmode") = 0, py::arg("bnact") = 0,
     py::arg("bnslope") = 0.f, py::arg("resbits") = 0, py::arg("resact") = 0, py::arg("resslope") = 0.f,
     py::arg("reflect") = 0, py::arg("ksplit") = 1, py::arg("ypart") = 0, py::arg("zfill") = 0, py::arg("bnx2") = 0,
     py::arg("bnprm2") = 0, py::arg("bnacc2") = 0, py::arg("w_ld") = 0, py::arg("w_kr") = 0, py::arg("w_ks") = 0);
  m.def("conv_fwd_variant", [](int v) { dv_conv_fwd_variant(v); });
  m.def("bn_tuning", [](int blocks, int unroll) { dv_bn_tuning(blocks, unroll); });
  m.def("bn_apply_tuning", [](int blocks, int unroll) { dv_bn_apply_tuning(blocks, unroll); });
  m.def("dw_variant", [](int v) { dv_dw_variant(v); });
  m.def("set_sync_check", [](bool on) { g_sync_check = on; });
  m.def("sync_check", []() { return g_sync_check; });
  m.def("set_deterministic", [](bool on) { dv_set_deterministic(on ? 1 : 0); });
  m.def("deterministic", []() { return dv_deterministic() != 0; });
  m.def("conv_wgrad_tuning", [](int v, int split_pct) { dv_conv_wgrad_tuning(v, split_pct); });
  m.def("conv_wgrad_slab", [](int mode) { dv_conv_wgrad_slab(mode); });
  // host-side split-K heuristic of conv_wgrad (no GPU work): tests pin the grid sizing
  m.def("conv_wgrad_splits", [](int Nb, int H, int W, int Cg, int Kout, int P_, int Q, int R, int S, int sh, int sw,
                                int ph, int pw) {
    ConvWgradArgs a{};
    a.Nb = Nb; a.H = H; a.W = W; a.Cg = Cg; a.ldx = Cg; a.G = 1; a.Kout = Kout; a.P = P_; a.Q = Q; a.ldy = Kout;
    a.R = R; a.S = S; a.sh = sh; a.sw = sw; a.ph = ph; a.pw = pw; a.dh = 1; a.dw_ = 1;
    return dv_conv_wgrad_splits(a);
  });
  m.def("conv_wgrad", [](uptr x, uptr dy, uptr dw, int Nb, int H, int W, int Cg, int ldx, int G, int Kout, int P_, int Q,
                         int ldy, int R, int S, int sh, int sw, int ph, int pw, int dh, int dwl, int splits, int accumulate,
                         int oirs_ig, uptr st, int reflect, uptr out, int out_ig, int out_accumulate) {
    ConvWgradArgs a{CP(x), CP(dy), FP(dw), Nb, H, W, Cg, ldx, G, Kout, P_, Q, ldy, R, S, sh, sw, ph, pw, dh, dwl, splits,
                    accumulate, oirs_ig, reflect, FP(out), out_ig, out_accumulate};
    int r = dv_conv_wgrad(a, ST(st));
    if (r < 0) throw std::runtime_error("conv_wgrad: unsupported geometry (channels must be a multiple of 8)");
    check_last("conv_wgrad");
    return r;
  }, py::arg("x"), py::arg("dy"), py::arg("dw"), py::arg("Nb"), py::arg("H"), py::arg("W"), py::arg("Cg"), py::arg("ldx"),
     py::arg("G"), py::arg("Kout"), py::arg("P"), py::arg("Q"), py::arg("ldy"), py::arg("R"), py::arg("S"), py::arg("sh"),
     py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("dh"), py::arg("dw_"), py::arg("splits"), py::arg("accumulate"),
     py::arg("oirs_ig"), py::arg("st"), py::arg("reflect") = 0, py::arg("out") = 0, py::arg("out_ig") = 0,
     py::arg("out_accumulate") = 0);
  m.attr("WGRAD_FINAL") = DV_WGRAD_FINAL;

  m.def("bn_stats", [](uptr x, int64_t rows, int C, uptr acc, uptr st) { dv_bn_stats(CP(x), rows, C, FP(acc), ST(st)); check_last("bn_stats"); });
  m.def("bn_finalize", [](uptr acc, int C, double count, float eps, float mom, uptr gamma, uptr beta, uptr rm, uptr rv,
                          uptr smean, uptr sinv, uptr scale, uptr shift, uptr st) {
    dv_bn_finalize(FP(acc), C, count, eps, mom, CFP(gamma), CFP(beta), FP(rm), FP(rv), FP(smean), FP(sinv), FP(scale), FP(shift), ST(st));
    check_last("bn_finalize");
  });
  m.def("bn_eval_prep", [](int C, float eps, uptr gamma, uptr beta, uptr rm, uptr rv, uptr scale, uptr shift, uptr st) {
    dv_bn_eval_prep(C, eps, CFP(gamma), CFP(beta), CFP(rm), CFP(rv), FP(scale), FP(shift), ST(st)); check_last("bn_eval_prep");
  });
  m.def("bn_apply", [](uptr x, uptr res, uptr out, int64_t n, int C, uptr scale, uptr shift, int act, float slope,
                       uptr mask, uptr st, uptr rscale, uptr rshift, int post) {
    dv_bn_apply(CP(x), CP(res), P(out), n, C, CFP(scale), CFP(shift), act, slope, P(mask), CFP(rscale), CFP(rshift), ST(st),
                post);
    check_last("bn_apply");
  }, py::arg("x"), py::arg("res"), py::arg("out"), py::arg("n"), py::arg("C"), py::arg("scale"), py::arg("shift"),
     py::arg("act"), py::arg("slope"), py::arg("mask"), py::arg("st"), py::arg("rscale") = 0, py::arg("rshift") = 0,
     py::arg("post") = 0);
  m.def("bn_fin_ok", [](int64_t n, int C) { return dv_bn_fin_ok(n, C); });
  m.def("bn_fin_apply", [](uptr acc, double count, float eps, float mom, uptr gamma, uptr beta, uptr rm, uptr rv, uptr prm,
                           uptr ticket, uptr x, uptr res, uptr out, int64_t n, int C, int act, float slope, uptr mask,
                           int post, uptr st) {
    dv_bn_fin_apply(FP(acc), count, eps, mom, CFP(gamma), CFP(beta), FP(rm), FP(rv), FP(prm), reinterpret_cast<int*>(ticket),
                    CP(x), CP(res), P(out), n, C, act, slope, P(mask), post, ST(st));
    check_last("bn_fin_apply");
  });
  m.def("bn_bwd_fin_apply", [](uptr acc, double count, uptr gamma, uptr mean, uptr invstd, uptr dgamma, uptr dbeta,
                               int accumulate, uptr xsum, uptr ticket, uptr dout, uptr out, uptr x, uptr dx, uptr dres,
                               int64_t n, int C, uptr mscale, uptr mshift, int act, float slope, int mask_bits, uptr addend,
                               uptr addend2, uptr colsum, uptr st) {
    dv_bn_bwd_fin_apply(FP(acc), count, CFP(gamma), CFP(mean), CFP(invstd), FP(dgamma), FP(dbeta), accumulate, FP(xsum),
                        reinterpret_cast<int*>(ticket), CP(dout), CP(out), CP(x), P(dx), P(dres), n, C, CFP(mscale),
                        CFP(mshift), act, slope, mask_bits, CP(addend), CP(addend2), FP(colsum), ST(st));
    check_last("bn_bwd_fin_apply");
  });
  m.def("bn_bwd_reduce", [](uptr dout, uptr out, uptr x, int64_t rows, int C, uptr mean, uptr invstd, uptr mscale,
                            uptr mshift, int act, float slope, uptr acc, int mask_bits, uptr st) {
    dv_bn_bwd_reduce(CP(dout), CP(out), CP(x), rows, C, CFP(mean), CFP(invstd), CFP(mscale), CFP(mshift), act, slope, FP(acc),
                     mask_bits, ST(st));
    check_last("bn_bwd_reduce");
  });
  m.def("bn_bwd_finalize", [](uptr acc, int C, double count, uptr gamma, uptr mean, uptr invstd, uptr dgamma, uptr dbeta,
                              int accumulate, uptr kA, uptr kB, uptr kC, uptr st, uptr xsum) {
    dv_bn_bwd_finalize(FP(acc), C, count, CFP(gamma), CFP(mean), CFP(invstd), FP(dgamma), FP(dbeta), accumulate, FP(kA), FP(kB), FP(kC), ST(st),
                       FP(xsum));
    check_last("bn_bwd_finalize");
  }, py::arg("acc"), py::arg("C"), py::arg("count"), py::arg("gamma"), py::arg("mean"), py::arg("invstd"), py::arg("dgamma"),
     py::arg("dbeta"), py::arg("accumulate"), py::arg("kA"), py::arg("kB"), py::arg("kC"), py::arg("st"), py::arg("xsum") = 0);
  m.def("bn_bwd_apply", [](uptr dout, uptr out, uptr x, uptr dx, uptr dres, int64_t n, int C, uptr kA, uptr kB, uptr kC,
                           uptr mscale, uptr mshift, int act, float slope, int mask_bits, uptr st, uptr addend, uptr addend2,
                           uptr colsum) {
    dv_bn_bwd_apply(CP(dout), CP(out), CP(x), P(dx), P(dres), n, C, CFP(kA), CFP(kB), CFP(kC), CFP(mscale), CFP(mshift), act, slope,
                    mask_bits, CP(addend), CP(addend2), FP(colsum), ST(st));
    check_last("bn_bwd_apply");
  }, py::arg("dout"), py::arg("out"), py::arg("x"), py::arg("dx"), py::arg("dres"), py::arg("n"), py::arg("C"), py::arg("kA"),
     py::arg("kB"), py::arg("kC"), py::arg("mscale"), py::arg("mshift"), py::arg("act"), py::arg("slope"),
     py::arg("mask_bits"), py::arg("st"), py::arg("addend") = 0, py::arg("addend2") = 0, py::arg("colsum") = 0);
  m.def("bn_bwd_apply_dual", [](uptr dout, uptr bits, uptr x, uptr x2, uptr dx, uptr dx2, int64_t n, int C, uptr k,
                                uptr k2, int act, float slope, uptr st) {
    if (C % 8 || n % C) throw std::runtime_error("bn_bwd_apply_dual: channels must be a multiple of 8");
    dv_bn_bwd_apply_dual(CP(dout), CP(bits), CP(x), CP(x2), P(dx), P(dx2), n, C, CFP(k), CFP(k2), act, slope, ST(st));
    check_last("bn_bwd_apply_dual");
  });
  m.def("bn_bwd_eval", [](uptr dout, uptr out, uptr dx, uptr dres, int64_t n, int C, uptr scale, int act, float slope, uptr st) {
    dv_bn_bwd_eval(CP(dout), CP(out), P(dx), P(dres), n, C, CFP(scale), act, slope, ST(st)); check_last("bn_bwd_eval");
  });

  m.def("maxpool_fwd", [](uptr x, uptr y, uptr idx, int N, int H, int W, int C, int P_, int Q, int kh, int kw, int sh, int sw,
                          int ph, int pw, uptr st, uptr stats) {
    const int r = dv_maxpool_fwd(CP(x), P(y), reinterpret_cast<uint8_t*>(idx), N, H, W, C, P_, Q, kh, kw, sh, sw, ph, pw,
                                 FP(stats), ST(st));
    check_last("maxpool_fwd");
    return r;
  }, py::arg("x"), py::arg("y"), py::arg("idx"), py::arg("N"), py::arg("H"), py::arg("W"), py::arg("C"), py::arg("P"),
     py::arg("Q"), py::arg("kh"), py::arg("kw"), py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("st"),
     py::arg("stats") = 0);
  m.def("maxpool_bwd", [](uptr dy, uptr idx, uptr dx, int N, int H, int W, int C, int P_, int Q, int kh, int kw, int sh,
                          int sw, int ph, int pw, uptr st) {
    dv_maxpool_bwd(CP(dy), reinterpret_cast<const uint8_t*>(idx), P(dx), N, H, W, C, P_, Q, kh, kw, sh, sw, ph, pw, ST(st)); check_last("maxpool_bwd");
  });
  m.def("bn_act_maxpool_fwd", [](uptr x, uptr y, uptr idx, int N, int H, int W, int C, int P_, int Q, int kh, int kw, int sh,
                                 int sw, int ph, int pw, uptr scale, uptr shift, int act, float slope, uptr st) {
    const int r = dv_bn_act_maxpool_fwd(CP(x), P(y), reinterpret_cast<uint8_t*>(idx), N, H, W, C, P_, Q, kh, kw, sh, sw, ph, pw,
                                        CFP(scale), CFP(shift), act, slope, ST(st));
    check_last("bn_act_maxpool_fwd");
    return r;
  });
  m.def("bn_act_maxpool_bwd", [](uptr dy, uptr idx, uptr x, uptr dx, int N, int H, int W, int C, int P_, int Q, int kh, int kw,
                                 int sh, int sw, int ph, int pw, uptr prm, uptr coef, int act, float slope, uptr acc, int apply,
                                 uptr st) {
    const int r = dv_bn_act_maxpool_bwd(CP(dy), reinterpret_cast<const uint8_t*>(idx), CP(x), P(dx), N, H, W, C, P_, Q, kh, kw,
                                        sh, sw, ph, pw, CFP(prm), CFP(coef), act, slope, FP(acc), apply, ST(st));
    check_last("bn_act_maxpool_bwd");
    return r;
  });
  m.def("avgpool_fwd", [](uptr x, uptr y, int N, int H, int W, int C, int P_, int Q, int kh, int kw, int sh, int sw, int ph,
                          int pw, int cip, int divover, uptr st) {
    dv_avgpool_fwd(CP(x), P(y), N, H, W, C, P_, Q, kh, kw, sh, sw, ph, pw, cip, divover, ST(st)); check_last("avgpool_fwd");
  });
  m.def("avgpool_bwd", [](uptr dy, uptr dx, int N, int H, int W, int C, int P_, int Q, int kh, int kw, int sh, int sw, int ph,
                          int pw, int cip, int divover, uptr st) {
    dv_avgpool_bwd(CP(dy), P(dx), N, H, W, C, P_, Q, kh, kw, sh, sw, ph, pw, cip, divover, ST(st)); check_last("avgpool_bwd");
  });
  m.def("gap_fwd", [](uptr x, uptr y, int N, int HW, int C, uptr st) { dv_gap_fwd(CP(x), P(y), N, HW, C, ST(st)); check_last("gap_fwd"); });
  m.def("gap_bwd", [](uptr dy, uptr dx, int N, int HW, int C, uptr st) { dv_gap_bwd(CP(dy), P(dx), N, HW, C, ST(st)); check_last("gap_bwd"); });
  m.def("upsample_fwd", [](uptr x, uptr y, int N, int H, int W, int C, int f, uptr st) { dv_upsample_fwd(CP(x), P(y), N, H, W, C, f, ST(st)); check_last("upsample_fwd"); });
  m.def("upsample_add", [](uptr x, uptr r, uptr y, int N, int H, int W, int C, int f, uptr st, uptr stats) {
    const int rc = dv_upsample_add(CP(x), CP(r), P(y), N, H, W, C, f, FP(stats), ST(st));
    check_last("upsample_add");
    return rc;
  }, py::arg("x"), py::arg("r"), py::arg("y"), py::arg("N"), py::arg("H"), py::arg("W"), py::arg("C"), py::arg("f"),
     py::arg("st"), py::arg("stats") = 0);
  m.def("upsample_bwd", [](uptr dy, uptr dx, int N, int H, int W, int C, int f, uptr st) { dv_upsample_bwd(CP(dy), P(dx), N, H, W, C, f, ST(st)); check_last("upsample_bwd"); });

  m.def("act_fwd", [](uptr x, uptr y, int64_t n, int act, float slope, uptr st) { dv_act_fwd(CP(x), P(y), n, act, slope, ST(st)); check_last("act_fwd"); });
  m.def("act_bwd", [](uptr dy, uptr y, uptr dx, int64_t n, int act, float slope, uptr st) { dv_act_bwd(CP(dy), CP(y), P(dx), n, act, slope, ST(st)); check_last("act_bwd"); });
  m.def("act_bwd_rows", [](uptr dy, int lddy, uptr y, int ldy, uptr dx, int lddx, int64_t rows, int C, int act, float slope,
                           uptr st) {
    if (dv_act_bwd_rows(CP(dy), lddy, CP(y), ldy, P(dx), lddx, rows, C, act, slope, ST(st)))
      throw std::runtime_error("act_bwd_rows: channel count / strides must be multiples of 8 and >= C");
    check_last("act_bwd_rows");
  });
  m.def("add", [](uptr a, uptr b, uptr y, int64_t n, float alpha, float beta, int act, float slope, uptr st) { dv_add(CP(a), CP(b), P(y), n, alpha, beta, act, slope, ST(st)); check_last("add"); });
  m.def("dropout", [](uptr x, uptr y, int64_t n, float p, uint64_t seed, uptr st, uptr step) {
    dv_dropout(CP(x), P(y), n, p, seed, (const uint32_t*)step, ST(st));
    check_last("dropout");
  }, py::arg("x"), py::arg("y"), py::arg("n"), py::arg("p"), py::arg("seed"), py::arg("st"), py::arg("step") = 0);
  m.def("wprep", [](uptr w, uptr out, int G, int Og, int Ig, int R, int S, int Ipad, int mode, int Sp, uptr st) { dv_wprep(CFP(w), P(out), G, Og, Ig, R, S, Ipad, mode, Sp, ST(st)); check_last("wprep"); });
  m.def("stem_fwd", [](uptr xp, uptr w, uptr y, uptr bias, uptr stats, int act, float slope, int N, int Hp, int Wp,
                       int P_, int Q, int R, int Sp, int K, int sh, int sw, uptr st) {
    const int r = dv_stem_fwd(CP(xp), CP(w), P(y), CFP(bias), FP(stats), act, slope, N, Hp, Wp, P_, Q, R, Sp, K, sh, sw,
                              ST(st));
    if (r == 0) check_last("stem_fwd");
    return r;
  });
  m.def("stem_wgrad", [](uptr xp, uptr dy, int ldy, uptr dw, int N, int C, int S, int Hp, int Wp, int P_, int Q, int R,
                         int Sp, int K, int sh, int sw, uptr st) {
    const int r = dv_stem_wgrad(CP(xp), CP(dy), ldy, FP(dw), N, C, S, Hp, Wp, P_, Q, R, Sp, K, sh, sw, ST(st));
    if (r == 0) check_last("stem_wgrad");
    return r;
  });
  m.def("stem_tuning", [](int blocks, int wg_blocks) { dv_stem_tuning(blocks, wg_blocks); });
  m.def("u8_jitter", [](uptr x, uptr prm, int N, int64_t npix, uptr st) {
    dv_u8_jitter(P(x), CFP(prm), N, npix, ST(st)); check_last("u8_jitter");
  });
  m.def("u8_normalize", [](uptr x, uptr flip, uptr y, int N, int C, int H, int W, float scale, std::vector<float> mean,
                           std::vector<float> sd, uptr st) {
    if (C < 1 || C > 3 || (int)mean.size() < C || (int)sd.size() < C) throw std::runtime_error("u8_normalize: 1-3 channels");
    dv_u8_normalize(CP(x), CP(flip), P(y), N, C, H, W, scale, mean.data(), sd.data(), ST(st)); check_last("u8_normalize");
  });
  m.def("stem_pack", [](uptr x, int is_f32, uptr y, int N, int C, int H, int W, int Hp, int Wp, int pt, int pl, uptr st,
                        int reflect) {
    dv_stem_pack(CP(x), is_f32, P(y), N, C, H, W, Hp, Wp, pt, pl, reflect, ST(st)); check_last("stem_pack");
  }, py::arg("x"), py::arg("is_f32"), py::arg("y"), py::arg("N"), py::arg("C"), py::arg("H"), py::arg("W"),
     py::arg("Hp"), py::arg("Wp"), py::arg("pt"), py::arg("pl"), py::arg("st"), py::arg("reflect") = 0);
  m.def("nhwc_copy", [](uptr src, int lds, uptr dst, int ldd, int64_t rows, int C, uptr idx, uptr st) {
    if (dv_nhwc_copy(CP(src), lds, P(dst), ldd, rows, C, (const int*)CP(idx), ST(st)))
      throw std::runtime_error("nhwc_copy: channel count / strides must be multiples of 8 for a plain copy");
    check_last("nhwc_copy");
  });
  m.def("reflect_pad_bwd", [](uptr dxp, uptr dx, int N, int H, int W, int C, int ldp, int ld, int ph, int pw, uptr st) {
    dv_reflect_pad_bwd(CP(dxp), P(dx), N, H, W, C, ldp, ld, ph, pw, ST(st)); check_last("reflect_pad_bwd");
  });
  m.def("wgrad_unprep", [](uptr src, uptr dst, int G, int Og, int Ig, int R, int S, int Ipad, float alpha, int accumulate,
                           int zero_src, uptr st) {
    dv_wgrad_unprep(FP(src), FP(dst), G, Og, Ig, R, S, Ipad, alpha, accumulate, zero_src, ST(st)); check_last("wgrad_unprep");
  });
  m.def("to_nhwc", [](uptr x, int is_f32, uptr y, int N, int C, int H, int W, int Cp, uptr st) { dv_to_nhwc(CP(x), is_f32, P(y), N, C, H, W, Cp, ST(st)); check_last("to_nhwc"); });
  m.def("f32_to_bf16", [](uptr x, uptr y, int64_t n, uptr st) { dv_f32_to_bf16(CFP(x), P(y), n, ST(st)); check_last("f32_to_bf16"); });

  m.def("scale_by", [](uptr in, uptr out, int64_t n, int is_bf16, uptr sp, uptr st) {
    dv_scale_by(CP(in), P(out), n, is_bf16, reinterpret_cast<const float*>(sp), ST(st));
    check_last("scale_by");
  });
  m.def("softmax_xent", [](uptr logits, int is_bf16, uptr labels, int rows, int C, uptr loss_rows, uptr grad, float gscale,
                           float ls, uptr st) {
    dv_softmax_xent(CP(logits), is_bf16, reinterpret_cast<const int64_t*>(labels), rows, C, FP(loss_rows), P(grad), gscale, ls, ST(st));
    check_last("softmax_xent");
  });
  m.def("sgd", [](uptr p, uptr g, uptr buf, int64_t n, float lr, float mom, float damp, float wd, int nesterov, int first,
                  float gscale, uptr st, uptr hp, uptr skip) {
    dv_sgd(FP(p), CFP(g), FP(buf), n, lr, mom, damp, wd, nesterov, first, gscale, CFP(hp), ST(st), CFP(skip)); check_last("sgd");
  }, py::arg("p"), py::arg("g"), py::arg("buf"), py::arg("n"), py::arg("lr"), py::arg("mom"), py::arg("damp"), py::arg("wd"),
     py::arg("nesterov"), py::arg("first"), py::arg("gscale"), py::arg("st"), py::arg("hp") = 0, py::arg("skip") = 0);
  m.def("adam", [](uptr p, uptr g, uptr mm, uptr v, int64_t n, float lr, float b1, float b2, float eps, float wd, int decoupled,
                   float bc1, float bc2, float gscale, uptr st, uptr hp, uptr skip) {
    dv_adam(FP(p), CFP(g), FP(mm), FP(v), n, lr, b1, b2, eps, wd, decoupled, bc1, bc2, gscale, CFP(hp), ST(st), CFP(skip));
    check_last("adam");
  }, py::arg("p"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("n"), py::arg("lr"), py::arg("b1"), py::arg("b2"),
     py::arg("eps"), py::arg("wd"), py::arg("decoupled"), py::arg("bc1"), py::arg("bc2"), py::arg("gscale"), py::arg("st"),
     py::arg("hp") = 0, py::arg("skip") = 0);
  m.def("rmsprop", [](uptr p, uptr g, uptr sq, uptr mom, uptr gavg, int64_t n, float lr, float alpha, float eps, float wd,
                      float momentum, int centered, float gscale, uptr st, uptr hp, uptr skip) {
    dv_rmsprop(FP(p), CFP(g), FP(sq), FP(mom), FP(gavg), n, lr, alpha, eps, wd, momentum, centered, gscale, CFP(hp), ST(st),
               CFP(skip));
    check_last("rmsprop");
  }, py::arg("p"), py::arg("g"), py::arg("sq"), py::arg("mom"), py::arg("gavg"), py::arg("n"), py::arg("lr"), py::arg("alpha"),
     py::arg("eps"), py::arg("wd"), py::arg("momentum"), py::arg("centered"), py::arg("gscale"), py::arg("st"),
     py::arg("hp") = 0, py::arg("skip") = 0);
  m.def("nonfinite_check", [](uptr g, int64_t n, uptr guard, uptr st) {
    dv_nonfinite_check(CFP(g), n, FP(guard), ST(st)); check_last("nonfinite_check");
  });
  m.def("nonfinite_tally", [](uptr guard, uptr st) { dv_nonfinite_tally(FP(guard), ST(st)); check_last("nonfinite_tally"); });
  m.def("gconv", [](uptr x, int ldx, int Cin, uptr tin, uptr w, int Orows, uptr y, int ldy, int Cout, uptr tout, int M,
                    int G, int Cg, int Og, int Kp, uptr stats, uptr st) {
    if (dv_gconv(CP(x), ldx, Cin, reinterpret_cast<const int16_t*>(tin), CP(w), Orows, P(y), ldy, Cout,
                 reinterpret_cast<const int16_t*>(tout), M, G, Cg, Og, Kp, FP(stats), ST(st)))
      throw std::runtime_error("gconv: unsupported shape");
    check_last("gconv");
  });
  m.def("gconv_wgrad", [](uptr x, int ldx, uptr tin, uptr dy, int ldy, uptr tout, uptr dw, int M, int G, int Cg, int Og,
                          uptr st) {
    if (dv_gconv_wgrad(CP(x), ldx, reinterpret_cast<const int16_t*>(tin), CP(dy), ldy,
                       reinterpret_cast<const int16_t*>(tout), FP(dw), M, G, Cg, Og, ST(st)))
      throw std::runtime_error("gconv_wgrad: unsupported shape");
    check_last("gconv_wgrad");
  });
  m.def("dw_fwd", [](uptr x, uptr w, uptr bias, uptr y, int N, int H, int W, int C, int ldx, int P_, int Q, int ldy, int K,
                     int sh, int sw, int ph, int pw, int act, float slope, uptr stats, uptr st) {
    if (dv_dw_fwd(CP(x), CFP(w), CFP(bias), P(y), N, H, W, C, ldx, P_, Q, ldy, K, sh, sw, ph, pw, act, slope, FP(stats), ST(st)))
      throw std::runtime_error("dw_fwd: unsupported shape");
    check_last("dw_fwd");
  });
  m.def("dw_dgrad", [](uptr dy, uptr w, uptr dx, int N, int H, int W, int C, int ldx, int P_, int Q, int ldy, int K, int sh,
                       int sw, int ph, int pw, uptr st, uptr bnx, uptr bnprm, uptr bnacc, int bnmode, int bnact,
                       float bnslope) {
    if (dv_dw_dgrad(CP(dy), CFP(w), P(dx), N, H, W, C, ldx, P_, Q, ldy, K, sh, sw, ph, pw, ST(st), CP(bnx), CFP(bnprm),
                    FP(bnacc), bnmode, bnact, bnslope))
      throw std::runtime_error("dw_dgrad: unsupported shape");
    check_last("dw_dgrad");
  }, py::arg("dy"), py::arg("w"), py::arg("dx"), py::arg("N"), py::arg("H"), py::arg("W"), py::arg("C"), py::arg("ldx"),
     py::arg("P"), py::arg("Q"), py::arg("ldy"), py::arg("K"), py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"),
     py::arg("st"), py::arg("bnx") = 0, py::arg("bnprm") = 0, py::arg("bnacc") = 0, py::arg("bnmode") = 0,
     py::arg("bnact") = 0, py::arg("bnslope") = 0.f);
  m.def("dw_wgrad", [](uptr x, uptr dy, uptr dw, int N, int H, int W, int C, int ldx, int P_, int Q, int ldy, int K, int sh,
                       int sw, int ph, int pw, int accumulate, uptr st) {
    if (dv_dw_wgrad(CP(x), CP(dy), FP(dw), N, H, W, C, ldx, P_, Q, ldy, K, sh, sw, ph, pw, accumulate, ST(st)))
      throw std::runtime_error("dw_wgrad: unsupported shape");
    check_last("dw_wgrad");
  });
  m.def("lrn_fwd", [](uptr x, uptr y, int64_t npix, int C, int lo, int hi, float alpha, float beta, float k, uptr st) {
    if (dv_lrn_fwd(CP(x), P(y), npix, C, lo, hi, alpha, beta, k, ST(st))) throw std::runtime_error("lrn_fwd: C > 1024");
    check_last("lrn_fwd");
  });
  m.def("lrn_bwd", [](uptr x, uptr dy, uptr dx, int64_t npix, int C, int lo, int hi, float alpha, float beta, float k, uptr st) {
    if (dv_lrn_bwd(CP(x), CP(dy), P(dx), npix, C, lo, hi, alpha, beta, k, ST(st))) throw std::runtime_error("lrn_bwd: C > 1024");
    check_last("lrn_bwd");
  });
  m.def("sumsq", [](uptr x, int64_t n, uptr out, uptr st) { dv_sumsq(CFP(x), n, FP(out), ST(st)); check_last("sumsq"); });

  m.def("channel_sum_finalize", [](uptr acc, int ld, int C, uptr out, int accumulate, uptr st) {
    dv_channel_sum_finalize(FP(acc), ld, C, FP(out), accumulate, ST(st));
    check_last("channel_sum_finalize");
  }, py::arg("acc"), py::arg("ld"), py::arg("C"), py::arg("out"), py::arg("accumulate"), py::arg("st"));
  m.def("channel_sum", [](uptr x, int64_t rows, int ld, int C, uptr acc, uptr out, int accumulate, uptr st) {
    dv_channel_sum(CP(x), rows, ld, C, FP(acc), FP(out), accumulate, ST(st));
    check_last("channel_sum");
  });
  m.def("yolo_encode", [](uptr boxes, uptr classes, int N, int B, int C, std::vector<float> anchors, uptr y0, uptr y1,
                          uptr y2, int g0, int g1, int g2, uptr st) {
    if (anchors.size() != 18) throw std::runtime_error("yolo_encode: 9 anchors (w, h) expected");
    dv_yolo_encode(CFP(boxes), reinterpret_cast<const int*>(classes), N, B, C, anchors.data(), FP(y0), FP(y1), FP(y2),
                   g0, g1, g2, ST(st));
    check_last("yolo_encode");
  });
  m.def("heatmaps", [](uptr px, uptr py, uptr vis, int N, int J, int H, int W, uptr out, uptr st) {
    dv_heatmaps(reinterpret_cast<const int*>(px), reinterpret_cast<const int*>(py), reinterpret_cast<const int*>(vis),
                N, J, H, W, FP(out), ST(st));
    check_last("heatmaps");
  });
  m.def("yolo_gather_boxes", [](uptr yt, int N, int cells, int D, uptr boxes, uptr counts, uptr st) {
    dv_yolo_gather_boxes(CFP(yt), N, cells, D, FP(boxes), reinterpret_cast<int*>(counts), ST(st));
    check_last("yolo_gather_boxes");
  });
  m.def("yolo_loss", [](uptr pred, int ldp, uptr yt, uptr boxes, uptr counts, uptr grad, uptr gw, uptr losses, int N, int g,
                        int C, std::vector<float> anchors, float grad_scale, float lambda_coord, float lambda_noobj,
                        float ignore_thresh, uptr st) {
    if (anchors.size() != 6) throw std::runtime_error("yolo_loss: 3 anchors (w, h) expected");
    dv_yolo_loss(CP(pred), ldp, CFP(yt), CFP(boxes), reinterpret_cast<const int*>(counts), P(grad), CFP(gw), FP(losses), N, g, C,
                 anchors.data(), grad_scale, lambda_coord, lambda_noobj, ignore_thresh, ST(st));
    check_last("yolo_loss");
  });
  m.def("yolo_decode", [](uptr pred, int ldp, int N, int g, int C, std::vector<float> anchors, uptr out, int rows_total,
                          int row_off, uptr st) {
    if (anchors.size() != 6) throw std::runtime_error("yolo_decode: 3 anchors (w, h) expected");
    dv_yolo_decode(CP(pred), ldp, N, g, C, anchors.data(), FP(out), rows_total, row_off, ST(st));
    check_last("yolo_decode");
  });
  m.def("nms", [](uptr cand, int N, int M, int D, float iou_thresh, float score_thresh, int max_det, uptr out, uptr st) {
    if (dv_nms(CFP(cand), N, M, D, iou_thresh, score_thresh, max_det, FP(out), ST(st)))
      throw std::runtime_error("nms: more than 32768 candidate rows per image");
    check_last("nms");
  });
  m.def("pw_loss", [](int kind, uptr pred, int pred_bf16, uptr tgt, int tgt_type, float tval, uptr wt, int64_t rows,
                      int C, int ldp, int ldt, float a, float b, uptr sums, uptr grad, uptr gscale, float hscale, uptr st) {
    dv_pw_loss(kind, CP(pred), pred_bf16, CP(tgt), tgt_type, tval, CFP(wt), rows, C, ldp, ldt, a, b, FP(sums), P(grad),
               CFP(gscale), hscale, ST(st));
    check_last("pw_loss");
  });
  m.def("wprep_batched", [](uptr descs, uptr chunks, int nchunks, uptr st) {
    dv_wprep_batched(CP(descs), CP(chunks), nchunks, ST(st));
    check_last("wprep_batched");
  });
  m.attr("WPREP_CHUNK") = WPREP_CHUNK;
  m.attr("WPREP_DESC_BYTES") = (int)sizeof(WprepDesc);
}
