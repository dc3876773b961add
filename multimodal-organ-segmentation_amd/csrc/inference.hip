// Sliding-window inference on device (reference trainer.py:370-395, which calls
// MONAI's sliding_window_inference with roi_size / overlap / sw_batch_size from
// configs/default.yaml:127-133; "mode" is not passed, so MONAI's default
// constant blending applies).
//
//   window_gather : windows [nw][M][r0][r1][r2] cut from the NCDHW volume,
//                   zero outside it (MONAI pads a volume smaller than the roi
//                   with zeros, symmetric; the host folds that padding into
//                   the window starts, which may be negative)
//   window_accum  : out[n][c][v] += logits of ONE window (launched per window
//                   in MONAI's window order, so every voxel's sum has the same
//                   fp32 addition order as MONAI's `output_image[idx] += pred`)
//   window_norm   : out /= count, count = per-axis coverage product (what
//                   MONAI's count_map holds for constant blending)
#include "mmseg_common.h"

namespace {

struct WinGeom {
  int N, C, D, H, W;     // volume (C = channels of the tensor being read / written)
  int r0, r1, r2;        // roi
};

__global__ void window_gather_kernel(const float* __restrict__ vol, WinGeom g, const int* __restrict__ win,
                                     int nw, float* __restrict__ out) {
  const long long rv = (long long)g.r0 * g.r1 * g.r2;
  const long long total = (long long)nw * g.C * rv;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(e % g.r2);
    long long q = e / g.r2;
    const int y = (int)(q % g.r1);
    q /= g.r1;
    const int z = (int)(q % g.r0);
    q /= g.r0;
    const int c = (int)(q % g.C);
    const int w = (int)(q / g.C);
    const int* s = win + 4 * w;    // (n, z0, y0, x0)
    const int zz = s[1] + z, yy = s[2] + y, xx = s[3] + x;
    float v = 0.f;
    if ((unsigned)zz < (unsigned)g.D && (unsigned)yy < (unsigned)g.H && (unsigned)xx < (unsigned)g.W)
      v = vol[(((long long)s[0] * g.C + c) * g.D + zz) * (long long)g.H * g.W + (long long)yy * g.W + xx];
    out[e] = v;
  }
}

__global__ void window_accum_kernel(const float* __restrict__ logits, WinGeom g, int n, int z0, int y0, int x0,
                                    float* __restrict__ out) {
  const long long rv = (long long)g.r0 * g.r1 * g.r2;
  const long long total = (long long)g.C * rv;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(e % g.r2);
    long long q = e / g.r2;
    const int y = (int)(q % g.r1);
    q /= g.r1;
    const int z = (int)(q % g.r0);
    const int c = (int)(q / g.r0);
    const int zz = z0 + z, yy = y0 + y, xx = x0 + x;
    if ((unsigned)zz < (unsigned)g.D && (unsigned)yy < (unsigned)g.H && (unsigned)xx < (unsigned)g.W) {
      float* o = out + (((long long)n * g.C + c) * g.D + zz) * (long long)g.H * g.W + (long long)yy * g.W + xx;
      *o = *o + logits[e];
    }
  }
}

__global__ void window_norm_kernel(float* __restrict__ out, WinGeom g, const float* __restrict__ cz,
                                   const float* __restrict__ cy, const float* __restrict__ cx) {
  const long long hw = (long long)g.H * g.W;
  const long long total = (long long)g.N * g.C * g.D * hw;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(e % g.W);
    const int y = (int)((e / g.W) % g.H);
    const int z = (int)((e / hw) % g.D);
    out[e] = out[e] / (cz[z] * cy[y] * cx[x]);
  }
}

int grid_for(long long total) {
  long long b = (total + 255) / 256;
  return (int)(b < 8192 ? (b < 1 ? 1 : b) : 8192);
}

}  // namespace

extern "C" {

int mmseg_window_gather(const float* vol, int N, int C, int D, int H, int W, const int* win, int nw, int r0, int r1,
                        int r2, float* out, void* stream) {
  MMSEG_REQUIRE(nw >= 1 && r0 > 0 && r1 > 0 && r2 > 0, "window_gather: empty window set");
  WinGeom g{N, C, D, H, W, r0, r1, r2};
  MMSEG_LAUNCH(window_gather_kernel, dim3(grid_for((long long)nw * C * r0 * r1 * r2)), dim3(256), 0,
                     (hipStream_t)stream, vol, g, win, nw, out);
  return mmseg::check_launch("window_gather");
}

int mmseg_window_accum(const float* logits, int N, int C, int D, int H, int W, int n, int z0, int y0, int x0, int r0,
                       int r1, int r2, float* out, void* stream) {
  MMSEG_REQUIRE(n >= 0 && n < N, "window_accum: sample %d out of range", n);
  WinGeom g{N, C, D, H, W, r0, r1, r2};
  MMSEG_LAUNCH(window_accum_kernel, dim3(grid_for((long long)C * r0 * r1 * r2)), dim3(256), 0,
                     (hipStream_t)stream, logits, g, n, z0, y0, x0, out);
  return mmseg::check_launch("window_accum");
}

int mmseg_window_norm(float* out, int N, int C, int D, int H, int W, const float* cz, const float* cy, const float* cx,
                      void* stream) {
  WinGeom g{N, C, D, H, W, 1, 1, 1};
  MMSEG_LAUNCH(window_norm_kernel, dim3(grid_for((long long)N * C * D * H * W)), dim3(256), 0,
                     (hipStream_t)stream, out, g, cz, cy, cx);
  return mmseg::check_launch("window_norm");
}

}  // extern "C"
