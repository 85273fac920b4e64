// Host-side entry points of every deep_vision_amd gfx950 kernel (called from bindings.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>

#define DV_STAT_SHARDS 64
// Forward BatchNorm statistics accumulator of C channels: [DV_STAT_SHARDS][2][C] shard partial
// sums of (x - K) and (x - K)^2, then one row [C] holding the per-channel shift K (the previous
// batch mean of that BN; csrc/bn.hip bn_finalize_kernel). Shifting keeps the single-pass
// variance free of E[x^2] - mean^2 cancellation when |mean| >> std.
#define DV_STAT_ROWS (2 * DV_STAT_SHARDS + 1)
static_assert(DV_STAT_SHARDS == 64, "common.h stat_shift() hard-codes the shard count");

struct ConvFwdArgs {
  const void* x;      // bf16 NHWC gathered tensor (input, or dY for dgrad)
  const void* w;      // bf16 [G][Kout][R][S][Cg]
  void* y;            // bf16 NHWC output
  const float* bias;  // [G*Kout] or nullptr
  float* stats;       // [tiles_m][2][G*Kout] or nullptr
  int Nb, H, W, Cg, ldx, G;
  int Kout, P, Q;     // GEMM columns per group, pixel grid enumerated by m
  int R, S, sh, sw, ph, pw, dh, dw;
  int tgather;        // 1: transposed-conv gather (dgrad with stride > 1); 2: tap-packed stem input
  int OH, OW, osh, osw, oph, opw, ldy;  // output pixel mapping
  int act; float slope;
  const void* res;    // optional residual added in the epilogue (layout of y, may alias y)
  // optional fused BatchNorm-backward statistics of the produced tensor (a dgrad whose output is
  // the incoming gradient of a BatchNorm): sum dz and sum dz*xhat per channel into bnacc
  const void* bnx;        // the BN's input (same layout as y)
  const void* bnbits;     // activation mask bits (bnmode 3) or nullptr
  const float* bnprm;     // [4][C]: scale, shift, mean, invstd
  float* bnacc;           // [SHARDS][2][C]
  int bnmode;             // 0 off, 1 no activation, 2 mask recomputed from bnx, 3 mask bits
  int bnact; float bnslope;
  // optional activation mask of `res` (1 bit per element, dense [rows][C/8] bytes): the epilogue
  // adds act'(res) -- res is the raw incoming gradient of a residual block's fused BN+add+ReLU
  // and the mask turns it into that block's shortcut gradient (no materialised dres tensor)
  const void* resbits;
  int resact; float resslope;
  // 1: out-of-image taps read the reflected pixel (ReflectionPad2d fused into the gather;
  // CycleGAN R/CycleGAN/tensorflow/models.py:8-14) instead of zeros
  int reflect;
  // split-K (short-M GEMMs such as Linear at batch 128: 25088->4096 is 32 tiles of 128x128 on
  // 256 CUs): ksplit > 1 splits the K loop over blocks; each split writes an fp32 slab
  // ypart[split][M][Kout] and a finalize pass sums the slabs in order, adds the bias, applies the
  // activation and writes bf16 y (deterministic; bias/act only, no statistics / residual / BN)
  int ksplit;
  float* ypart;
  // 1: strided output map (osh/osw > 1, no offset) of a scatter-form dgrad: every stored chunk
  // also zeroes the (osh x osw) - 1 output pixels its tap never reaches, so the output needs no
  // separate zero fill (1x1 stride-s dgrad: every pixel of the input grid is written once)
  int zfill = 0;
  // optional second BatchNorm fed by the same dz (a residual block's projection-shortcut BN folded
  // into the block's last BN pass: both see act'(z) * dout with the bnmode-3 mask): its input,
  // [4][C] parameters and accumulator. The sum dz is shared, the sum dz*xhat is its own.
  const void* bnx2 = nullptr;
  const float* bnprm2 = nullptr;
  float* bnacc2 = nullptr;
  // weight operand layout (fast loader only): elements between output-channel rows (0 = R*S*Cg)
  // and between consecutive taps of a row / column (0 = S*Cg / Cg). A tap subset of a larger
  // filter reads the full cached weight in place: w points at its first tap (sub-pixel dgrad)
  int w_ld = 0, w_kr = 0, w_ks = 0;
};

struct ConvWgradArgs {
  const void* x;   // bf16 NHWC forward input (im2col source)
  const void* dy;  // bf16 NHWC gradient of the output
  float* dw;       // fp32 [G][Kout][R][S][Cg]
  int Nb, H, W, Cg, ldx, G;
  int Kout, P, Q, ldy;
  int R, S, sh, sw, ph, pw, dh, dw_;
  int splits;      // 0 = heuristic
  int accumulate;  // add into dw (live gradient buffer) instead of overwriting
  int oirs_ig;     // > 0: dw is the parameter's own [G*Kout][oirs_ig][R][S] layout (padded channels dropped)
  int reflect;     // im2col with reflected out-of-image taps (see ConvFwdArgs)
  // optional: the parameter's OIHW gradient [G*Kout][out_ig][R][S]. When the split-K partials go
  // through ordered slabs, their reduce pass writes (or with out_accumulate adds) straight into it
  // and dv_conv_wgrad returns splits | DV_WGRAD_FINAL; otherwise `dw` holds the packed result.
  float* out;
  int out_ig, out_accumulate;
};
constexpr int DV_WGRAD_FINAL = 1 << 30;

int dv_conv_fwd(const ConvFwdArgs& a, hipStream_t st);  // 0 ok, 1 ok but BN statistics not fused, -1 unsupported
void dv_conv_fwd_variant(int v);  // 0 = heuristic tile choice; others: benchmarking override
int dv_conv_wgrad(const ConvWgradArgs& a, hipStream_t st);
// grouped 1x1 conv with small unaligned groups and a fused channel shuffle (csrc/gconv.hip):
// forward / dgrad (weights [G][Orows][Kp] bf16) and the fp32 weight gradient (accumulated);
// tin / tout: logical -> stored channel tables (int16, nullptr = identity)
int dv_gconv(const void* x, int ldx, int Cin, const int16_t* tin, const void* w, int Orows, void* y, int ldy, int Cout,
             const int16_t* tout, int M, int G, int Cg, int Og, int Kp, float* stats, hipStream_t st);
int dv_gconv_wgrad(const void* x, int ldx, const int16_t* tin, const void* dy, int ldy, const int16_t* tout, float* dw,
                   int M, int G, int Cg, int Og, hipStream_t st);
void dv_conv_wgrad_tuning(int variant, int split_pct);  // benchmarking override (0, 100 = heuristic)
void dv_conv_wgrad_slab(int on);  // split-K combine: -1 auto (slabs up to 64 splits), 1 ordered fp32 slabs, 0 float atomics
int dv_conv_wgrad_splits(const ConvWgradArgs& a);
// deterministic mode: split-K weight gradients go through per-split fp32 slabs reduced in a
// fixed order instead of atomics (bitwise-reproducible dW)
void dv_set_deterministic(int on);
int dv_deterministic();
// shared fp32 slab workspace (grown on demand) and the fixed-order slab sum
// dst[i] (+)= sum_{s < splits} ws[s * n + i] used by every deterministic weight gradient
float* dv_slab_workspace(size_t elems, hipStream_t st);
// Deterministic BatchNorm statistics: a statistics-producing launch with `rows` reduction blocks
// writes each block's [2][ncols] partial row into its own row of a zeroed per-stream slab
// (common.h stat_row) instead of atomics into shard blk % 64; fold() then adds the slab rows, in
// a fixed order, into the accumulator's 64 shards (and re-zeroes the slab). Off (slab == nullptr,
// fold() a no-op) unless dv_deterministic().
float* dv_det_workspace(size_t elems, hipStream_t st);
void dv_det_fold(float* slab, int64_t rows, int64_t width, float* acc, int64_t stride, hipStream_t st);
// scalar-ish sums (loss totals): dst[j] += sum_r slab[r][j] in a fixed order, slab re-zeroed
void dv_det_sum(float* slab, int64_t rows, int64_t width, float* dst, hipStream_t st);
struct DetStats {
  float* slab = nullptr;
  int64_t rows = 0, width = 0;
  hipStream_t st = nullptr;
  DetStats(int64_t rows_, int64_t ncols, hipStream_t st_, int regions = 1) : rows(rows_), width(2 * ncols), st(st_) {
    if (dv_deterministic() && rows > 0) slab = dv_det_workspace((size_t)(rows * width * regions), st);
  }
  float* region(int i) const { return slab ? slab + (int64_t)i * rows * width : nullptr; }
  // shards of acc are [64][2][ncols]: row stride = width
  void fold(float* acc, int i = 0) const {
    if (slab && acc) dv_det_fold(region(i), rows, width, acc, width, st);
  }
};
void dv_slab_reduce(const float* ws, float* dst, int64_t n, int splits, int accumulate, hipStream_t st);
int dv_conv_stats_tiles(int Nb, int P, int Q);

// ---- batchnorm (bn.hip) ----
void dv_bn_tuning(int reduce_blocks, int reduce_unroll);  // benchmarking override (1024, 2 = default)
void dv_bn_apply_tuning(int blocks, int unroll);          // apply passes: benchmarking override (4096, 2)
void dv_bn_stats(const void* x, int64_t rows, int C, float* acc, hipStream_t st);
void dv_bn_finalize(float* acc, int C, double count, float eps, float momentum, const float* gamma,
                    const float* beta, float* rm, float* rv, float* save_mean, float* save_invstd, float* scale,
                    float* shift, hipStream_t st);
// Small BatchNorms (C % 64 == 0, at most DV_BN_FIN_MAX_ELEMS elements): the statistics fold inside
// the apply pass, no finalize launch (bn.hip "Small BatchNorms"). ticket: [C / 64] zeroed ints.
#define DV_BN_FIN_MAX_ELEMS (2ll << 20)
bool dv_bn_fin_ok(int64_t n, int C);
void dv_bn_fin_apply(float* acc, double count, float eps, float momentum, const float* gamma, const float* beta,
                     float* rm, float* rv, float* prm, int* ticket, const void* x, const void* res, void* out, int64_t n,
                     int C, int act, float slope, void* mask, int post, hipStream_t st);
void dv_bn_bwd_fin_apply(float* acc, double count, const float* gamma, const float* mean, const float* invstd,
                         float* dgamma, float* dbeta, int accumulate, float* xsum, int* ticket, const void* dout,
                         const void* out, const void* x, void* dx, void* dres, int64_t n, int C, const float* mscale,
                         const float* mshift, int act, float slope, int mask_bits, const void* addend,
                         const void* addend2, float* colsum, hipStream_t st);
void dv_bn_eval_prep(int C, float eps, const float* gamma, const float* beta, const float* rm, const float* rv,
                     float* scale, float* shift, hipStream_t st);
// out = act(x*scale + shift (+ res [* rscale + rshift])): rscale/rshift fold a second BatchNorm
// (a residual block's projection BN) into the same pass instead of materialising its output
void dv_bn_apply(const void* x, const void* res, void* out, int64_t n, int C, const float* scale, const float* shift,
                 int act, float slope, void* mask, const float* rscale, const float* rshift, hipStream_t st, int post = 0);
void dv_bn_bwd_reduce(const void* dout, const void* out, const void* x, int64_t rows, int C, const float* mean,
                      const float* invstd, const float* mscale, const float* mshift, int act, float slope, float* acc,
                      int mask_bits, hipStream_t st);
void dv_bn_bwd_finalize(float* acc, int C, double count, const float* gamma, const float* mean, const float* invstd,
                        float* dgamma, float* dbeta, int accumulate, float* kA, float* kB, float* kC, hipStream_t st,
                        float* xsum = nullptr);
void dv_bn_bwd_apply(const void* dout, const void* out, const void* x, void* dx, void* dres, int64_t n, int C,
                     const float* kA, const float* kB, const float* kC, const float* mscale, const float* mshift, int act,
                     float slope, int mask_bits, const void* addend, const void* addend2, float* colsum,
                     hipStream_t st);
// both BatchNorms of a residual block's output join (main + folded projection BN, one mask):
// dz = act'(z)*dout from the mask bits, dx = kA*dz + kB*x + kC, dx2 = kA2*dz + kB2*x2 + kC2
void dv_bn_bwd_apply_dual(const void* dout, const void* bits, const void* x, const void* x2, void* dx, void* dx2,
                          int64_t n, int C, const float* k, const float* k2, int act, float slope, hipStream_t st);
void dv_bn_bwd_eval(const void* dout, const void* out, void* dx, void* dres, int64_t n, int C, const float* scale,
                    int act, float slope, hipStream_t st);

// ---- pooling (pool.hip) ----
// stats: fused BatchNorm statistics of y into a [SHARDS][2][C] + shift accumulator (-1: unsupported C)
int dv_maxpool_fwd(const void* x, void* y, uint8_t* idx, int N, int H, int W, int C, int P, int Q, int kh, int kw,
                   int sh, int sw, int ph, int pw, float* stats, hipStream_t st);
void dv_maxpool_bwd(const void* dy, const uint8_t* idx, void* dx, int N, int H, int W, int C, int P, int Q, int kh,
                    int kw, int sh, int sw, int ph, int pw, hipStream_t st);
// fused BatchNorm apply + activation + max pool (ResNet stem); -1 = shape not covered
int dv_bn_act_maxpool_fwd(const void* x, void* y, uint8_t* idx, int N, int H, int W, int C, int P, int Q, int kh, int kw,
                          int sh, int sw, int ph, int pw, const float* scale, const float* shift, int act, float slope,
                          hipStream_t st);
int dv_bn_act_maxpool_bwd(const void* dy, const uint8_t* idx, const void* x, void* dx, int N, int H, int W, int C, int P,
                          int Q, int kh, int kw, int sh, int sw, int ph, int pw, const float* prm, const float* coef,
                          int act, float slope, float* acc, int apply, hipStream_t st);
void dv_avgpool_fwd(const void* x, void* y, int N, int H, int W, int C, int P, int Q, int kh, int kw, int sh, int sw,
                    int ph, int pw, int cip, int divover, hipStream_t st);
void dv_avgpool_bwd(const void* dy, void* dx, int N, int H, int W, int C, int P, int Q, int kh, int kw, int sh, int sw,
                    int ph, int pw, int cip, int divover, hipStream_t st);
void dv_gap_fwd(const void* x, void* y, int N, int HW, int C, hipStream_t st);
void dv_gap_bwd(const void* dy, void* dx, int N, int HW, int C, hipStream_t st);
void dv_upsample_fwd(const void* x, void* y, int N, int H, int W, int C, int f, hipStream_t st);
int dv_upsample_add(const void* x, const void* r, void* y, int N, int H, int W, int C, int f, float* stats,
                    hipStream_t st);
void dv_upsample_bwd(const void* dy, void* dx, int N, int H, int W, int C, int f, hipStream_t st);

// ---- elementwise / layout (elementwise.hip) ----
void dv_act_fwd(const void* x, void* y, int64_t n, int act, float slope, hipStream_t st);
void dv_act_bwd(const void* dy, const void* y, void* dx, int64_t n, int act, float slope, hipStream_t st);
// strided rows x C form (each tensor its own pixel stride); -1 when strides / C are not multiples of 8
int dv_act_bwd_rows(const void* dy, int lddy, const void* y, int ldy, void* dx, int lddx, int64_t rows, int C, int act,
                    float slope, hipStream_t st);
void dv_add(const void* a, const void* b, void* y, int64_t n, float alpha, float beta, int act, float slope, hipStream_t st);
void dv_dropout(const void* x, void* y, int64_t n, float p, uint64_t seed, const uint32_t* step, hipStream_t st);
void dv_wprep(const float* w, void* out, int G, int Og, int Ig, int R, int S, int Ipad, int mode, int Sp, hipStream_t st);
// NHWC channel-slice copy (16-B vectors; concat into a slice of a wider buffer) or, with an index
// table, a channel gather (ShuffleNet channel shuffle / its inverse). -1: unsupported geometry.
int dv_nhwc_copy(const void* src, int lds, void* dst, int ldd, int64_t rows, int C, const int* idx, hipStream_t st);
// reflection-pad backward: dx[h][w] = sum of the padded gradient at every padded position that
// reflects onto (h, w) (the interior one plus up to three mirrored border positions)
void dv_reflect_pad_bwd(const void* dxp, void* dx, int N, int H, int W, int C, int ldp, int ld, int ph, int pw,
                        hipStream_t st);
// dedicated 7x7 / 64-channel stem kernels on the tap-packed image (csrc/stem.hip); -1 = not covered
int dv_stem_fwd(const void* xp, const void* w, void* y, const float* bias, float* stats, int act, float slope, int N,
                int Hp, int Wp, int P, int Q, int R, int Sp, int K, int sh, int sw, hipStream_t st);
int dv_stem_wgrad(const void* xp, const void* dy, int ldy, float* dw, int N, int C, int S, int Hp, int Wp, int P, int Q,
                  int R, int Sp, int K, int sh, int sw, hipStream_t st);
void dv_stem_tuning(int blocks, int wg_blocks);  // benchmarking override of the target grids (0 = default)
void dv_stem_pack(const void* x, int x_is_f32, void* y, int N, int C, int H, int W, int Hp, int Wp, int pt, int pl,
                  int reflect, hipStream_t st);
void dv_wgrad_unprep(float* src, float* dst, int G, int Og, int Ig, int R, int S, int Ipad, float alpha,
                     int accumulate, int zero_src, hipStream_t st);
void dv_to_nhwc(const void* x, int x_is_f32, void* y, int N, int C, int H, int W, int Cp, hipStream_t st);
// uint8 HWC input crops -> normalised bf16 NCHW (C <= 3, host mean / std), optional per-sample flip
void dv_u8_jitter(void* x, const float* prm, int N, int64_t npix, hipStream_t st);
void dv_u8_normalize(const void* x, const void* flip, void* y, int N, int C, int H, int W, float scale, const float* mean,
                     const float* std_, hipStream_t st);
void dv_f32_to_bf16(const float* x, void* y, int64_t n, hipStream_t st);

// ---- loss / optimizers (loss_optim.hip) ----
void dv_scale_by(const void* in, void* out, int64_t n, int is_bf16, const float* s, hipStream_t st);
void dv_softmax_xent(const void* logits, int is_bf16, const int64_t* labels, int rows, int C, float* loss_rows, void* grad,
                     float grad_scale, float label_smoothing, hipStream_t st);
void dv_sgd(float* p, const float* g, float* buf, int64_t n, float lr, float momentum, float dampening, float wd,
            int nesterov, int first, float gscale, const float* hp, hipStream_t st, const float* skip = nullptr);
void dv_adam(float* p, const float* g, float* m, float* v, int64_t n, float lr, float b1, float b2, float eps, float wd,
             int decoupled, float bc1, float bc2, float gscale, const float* hp, hipStream_t st,
             const float* skip = nullptr);
void dv_rmsprop(float* p, const float* g, float* sq, float* mom, float* gavg, int64_t n, float lr, float alpha, float eps,
                float wd, float momentum, int centered, float gscale, const float* hp, hipStream_t st,
                const float* skip = nullptr);
void dv_nonfinite_check(const float* g, int64_t n, float* guard, hipStream_t st);
void dv_nonfinite_tally(float* guard, hipStream_t st);
void dv_sumsq(const float* x, int64_t n, float* out, hipStream_t st);

// ---- depthwise conv (depthwise.hip) ----
void dv_dw_variant(int v);  // benchmarking override of strip length / occupancy (0 = heuristic)
int dv_dw_fwd(const void* x, const float* w, const float* bias, void* y, int N, int H, int W, int C, int ldx, int P,
              int Q, int ldy, int K, int sh, int sw, int ph, int pw, int act, float slope, float* stats, hipStream_t st);
// bnmode 1 / 2: also reduce the BatchNorm-backward sums of dx (dx is that BN's output gradient)
// into bnacc, as the MFMA dgrad epilogues do (see ConvFwdArgs); -1 when the fusion cannot apply
int dv_dw_dgrad(const void* dy, const float* w, void* dx, int N, int H, int W, int C, int ldx, int P, int Q, int ldy,
                int K, int sh, int sw, int ph, int pw, hipStream_t st, const void* bnx = nullptr,
                const float* bnprm = nullptr, float* bnacc = nullptr, int bnmode = 0, int bnact = 0, float bnslope = 0.f);
int dv_dw_wgrad(const void* x, const void* dy, float* dw, int N, int H, int W, int C, int ldx, int P, int Q, int ldy,
                int K, int sh, int sw, int ph, int pw, int accumulate, hipStream_t st);

// ---- local response normalisation (lrn.hip) ----
int dv_lrn_fwd(const void* x, void* y, int64_t npix, int C, int lo, int hi, float alpha, float beta, float k,
               hipStream_t st);
int dv_lrn_bwd(const void* x, const void* dy, void* dx, int64_t npix, int C, int lo, int hi, float alpha, float beta,
               float k, hipStream_t st);

// ---- YOLOv3 head: loss + grad, decode, NMS (yolo.hip) ----
void dv_yolo_gather_boxes(const float* y_true, int N, int cells, int D, float* boxes, int* counts, hipStream_t st);
void dv_yolo_loss(const void* pred, int ldp, const float* y_true, const float* boxes, const int* counts, void* grad,
                  const float* gw, float* losses, int N, int g, int C, const float* anchors6, float grad_scale, float lambda_coord,
                  float lambda_noobj, float ignore_thresh, hipStream_t st);
void dv_yolo_decode(const void* pred, int ldp, int N, int g, int C, const float* anchors6, float* out, int rows_total,
                    int row_off, hipStream_t st);
int dv_nms(const float* cand, int N, int M, int D, float iou_thresh, float score_thresh, int max_det, float* out,
           hipStream_t st);

// ---- pointwise losses with gradient (losses.hip) ----
void dv_pw_loss(int kind, const void* pred, int pred_bf16, const void* tgt, int tgt_type, float tval, const float* wt,
                int64_t rows, int C, int ldp, int ldt, float a, float b, float* sums, void* grad, const float* gscale,
                float hscale, hipStream_t st);

// ---- batched weight prep (elementwise.hip) ----
#define WPREP_CHUNK 4096
struct WprepDesc {  // 48 bytes, mirrored by deep_vision_amd/ops/wcache.py
  const float* w;
  unsigned short* out;
  int64_t total;
  int G, Og, Ig, R, S, pad, mode, Sp;  // Sp: padded filter width (mode 2)
};
void dv_wprep_batched(const void* descs, const void* chunks, int nchunks, hipStream_t st);

// ---- training targets on the device (csrc/labels.hip) ----
// YOLOv3: boxes (N, B, 4) x1y1x2y2 normalised, classes (N, B) int (-1 = padding), anchors 9 x (w, h);
// y0/y1/y2 (N, g, g, 3, 5 + C) fp32, zeroed by the caller
void dv_yolo_encode(const float* boxes, const int* classes, int N, int B, int C, const float* anchors_wh, float* y0,
                    float* y1, float* y2, int g0, int g1, int g2, hipStream_t st);
// Stacked Hourglass: integer keypoint coordinates px/py and visibility (N, J) -> out (N, J, H, W) fp32
void dv_heatmaps(const int* px, const int* py, const int* vis, int N, int J, int H, int W, float* out, hipStream_t st);
// per-channel fp32 sum of a bf16 [rows][ld] tensor into out[C] (accumulate: +=); acc is a
// zeroed [SHARDS][2][ld] workspace that the call leaves zeroed
void dv_channel_sum(const void* x, int64_t rows, int ld, int C, float* acc, float* out, int accumulate, hipStream_t st);
// the fold half of dv_channel_sum: shards (filled by a fused producer, e.g. dv_bn_bwd_apply colsum) -> out
void dv_channel_sum_finalize(float* acc, int ld, int C, float* out, int accumulate, hipStream_t st);
