// On-device training-target construction: the reference builds these in tf.data
// on the CPU (R/YOLO/tensorflow/preprocess.py:137-224 label encoding,
// R/Hourglass/tensorflow/preprocess.py:91-173 Gaussian heatmaps); at 8 GPUs x 16 YOLO images per
// step the host encoder would feed ~2.7 MB of mostly-zero fp32 targets per image through the
// loader workers and the PCIe link. Here the loader ships only the raw ground truth (<= 100 boxes
// or 16 keypoints per image) and the targets are written straight into device memory.
#include "common.h"
#include "kernels.h"

// bit-for-bit the numpy float32 expressions: no a*b+c contraction into an FMA
#pragma clang fp contract(off)

namespace {

struct Anchors9 {
  float wh[18];  // 9 (w, h) pairs, normalised to the input size
};

// One block per image. Every thread walks the image's boxes in order and owns the target
// channels t = threadIdx.x, +blockDim.x, ... of whatever (cell, anchor) row the box lands in, so
// a later box that hits the same row overwrites it entirely (the last-writer-wins semantics of
// tensor_scatter_nd_update / the numpy encoder, data/yolo.py) with no cross-thread ordering.
// Targets must be zeroed by the caller: (N, g, g, 3, 5 + C) fp32 for the three grids.
__global__ __launch_bounds__(128) void yolo_encode_kernel(const float* __restrict__ boxes, const int* __restrict__ classes,
                                                          int B, int C, Anchors9 an, float* __restrict__ y0,
                                                          float* __restrict__ y1, float* __restrict__ y2, int g0, int g1,
                                                          int g2) {
  const int n = blockIdx.x;
  const int D = 5 + C;
  for (int b = 0; b < B; ++b) {
    const int cls = classes[(int64_t)n * B + b];
    if (cls < 0) continue;  // padding
    const float* bx = boxes + ((int64_t)n * B + b) * 4;
    const float x1 = bx[0], y1v = bx[1], x2 = bx[2], y2v = bx[3];
    const float w = x2 - x1, h = y2v - y1v;
    // best anchor by width/height IoU; first maximum wins (np.argmax)
    int best = 0;
    float bi = -1.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const float aw = an.wh[2 * k], ah = an.wh[2 * k + 1];
      const float inter = fminf(w, aw) * fminf(h, ah);
      const float iou = inter / (w * h + aw * ah - inter);
      if (iou > bi) { bi = iou; best = k; }
    }
    const int s = best / 3, a = best - s * 3;
    const int g = s == 0 ? g0 : (s == 1 ? g1 : g2);
    float* y = s == 0 ? y0 : (s == 1 ? y1 : y2);
    const float cx = (x1 + x2) / 2.f, cy = (y1v + y2v) / 2.f;
    const float cellw = 1.f / (float)g;
    const int ix = min(max((int)floorf(cx / cellw), 0), g - 1);
    const int iy = min(max((int)floorf(cy / cellw), 0), g - 1);
    float* row = y + ((((int64_t)n * g + iy) * g + ix) * 3 + a) * D;
    for (int t = threadIdx.x; t < D; t += blockDim.x) {
      float v;
      if (t == 0) v = cx;
      else if (t == 1) v = cy;
      else if (t == 2) v = w;
      else if (t == 3) v = h;
      else if (t == 4) v = 1.f;
      else v = (t - 5 == cls) ? 1.f : 0.f;
      row[t] = v;
    }
  }
}

// Stacked-Hourglass targets: out[n][j][y][x] = 12 * exp(-((x-x0)^2 + (y-y0)^2) / 2) inside the
// reference's 7x7 patch window [x0-3, x0+3) x [y0-3, y0+3) (its patch bounds exclude the last
// row / column), zero elsewhere and for invisible joints. (x0, y0) are the integer heatmap
// coordinates (the host rounds the float64 keypoints half-to-even like np.round); exp in double
// as numpy evaluates it, then rounded to fp32.
__global__ __launch_bounds__(256) void heatmap_kernel(const int* __restrict__ px, const int* __restrict__ py,
                                                      const int* __restrict__ vis, int J, int H, int W,
                                                      float* __restrict__ out) {
  const int j = blockIdx.y, n = blockIdx.z;
  const int pix = blockIdx.x * 256 + threadIdx.x;
  if (pix >= H * W) return;
  const int y = pix / W, x = pix - y * W;
  const int64_t k = (int64_t)n * J + j;
  const int x0 = px[k], y0 = py[k];
  const int xmin = x0 - 3, ymin = y0 - 3, xmax = x0 + 3, ymax = y0 + 3;
  float v = 0.f;
  const bool empty = xmin >= W || ymin >= H || xmax < 0 || ymax < 0 || vis[k] == 0;
  if (!empty && x >= xmin && x < xmax && y >= ymin && y < ymax) {
    const double dx = x - x0, dy = y - y0;
    v = (float)(exp(-(dx * dx + dy * dy) / 2.0) * 12.0);
  }
  out[(k * H + y) * W + x] = v;
}

}  // namespace

void dv_yolo_encode(const float* boxes, const int* classes, int N, int B, int C, const float* anchors_wh, float* y0,
                    float* y1, float* y2, int g0, int g1, int g2, hipStream_t st) {
  Anchors9 an;
  for (int i = 0; i < 18; ++i) an.wh[i] = anchors_wh[i];
  if (N <= 0) return;
  yolo_encode_kernel<<<dim3(N), dim3(128), 0, st>>>(boxes, classes, B, C, an, y0, y1, y2, g0, g1, g2);
}

void dv_heatmaps(const int* px, const int* py, const int* vis, int N, int J, int H, int W, float* out, hipStream_t st) {
  if (N <= 0 || J <= 0) return;
  heatmap_kernel<<<dim3((H * W + 255) / 256, J, N), dim3(256), 0, st>>>(px, py, vis, J, H, W, out);
}
