// Register-staged A-transform launches of the implicit-GEMM convolution (kernels.h ConvFwdArgs
// at_*): a deferred BatchNorm apply folded into a 1x1 conv / dgrad operand load (ops/defer.py).
#include "conv_fwd_core.h"

void dv_conv_fwd_at(const dvconv::FwdParams& p, int at, hipStream_t st) {
  switch (at) {
    case AT_BN: dispatch_at<AT_BN>(p, st); break;
    case AT_JOIN: dispatch_at<AT_JOIN>(p, st); break;
    case AT_BWDB: dispatch_at<AT_BWDB>(p, st); break;
    default: dispatch_at<AT_BWDX>(p, st); break;
  }
}
