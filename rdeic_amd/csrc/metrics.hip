// Full-reference image quality on the device: SSIM and MS-SSIM of uint8 RGB reconstructions
// against their originals, as the reference's evaluation reports them (pyiqa "ssim" / "ms_ssim",
// experiments/run_robustness.py:70-83, inference_partition.py:46-58; pyiqa is not in this image,
// so the algorithm is restated from its published definition — parity unpinned):
//
//   * test_y_channel: Y = round(255 * (0.299 R + 0.587 G + 0.114 B)) with R, G, B in [0, 1]
//     (YIQ luma, rounded half-to-even), data_range 255;
//   * SSIM (Wang et al. 2004): 11x11 Gaussian window, sigma 1.5, 'valid' filtering,
//     C1 = (0.01 * 255)^2, C2 = (0.03 * 255)^2, cs = relu((2 s12 + C2) / (s11 + s22 + C2)),
//     ssim = (2 mu1 mu2 + C1) / (mu1^2 + mu2^2 + C1) * cs, averaged over the valid pixels;
//   * MS-SSIM: 5 levels with weights (0.0448, 0.2856, 0.3001, 0.2363, 0.1333), 2x2 average
//     pooling between levels, prod_{l<4} cs_l^w_l * ssim_4^w_4 (the host combines the level means).
//
// The Gaussian is applied separably (horizontal pass into LDS, then vertical), one block per
// 64 x 16 tile of valid outputs; block sums go to a partial buffer and a finalize kernel adds
// them in a fixed order (fp64), so the result is deterministic.
#include <algorithm>
#include <cmath>

#include "common.h"
#include "../../include/rdeic_hip.h"

namespace {

constexpr int SS_W = 11, SS_R = 5;      // window, radius
constexpr int SS_TW = 64, SS_TH = 16;   // valid outputs per block
constexpr int SS_IW = SS_TW + 2 * SS_R, SS_IH = SS_TH + 2 * SS_R;

struct SsimWin { float g[SS_W]; };

// Y of one RGB u8 image pair (two planes) and the pyramid level-0 copies
__global__ __launch_bounds__(256) void rgb_to_y_kernel(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b,
                                                       long npix, float* __restrict__ ya, float* __restrict__ yb) {
  const long img = blockIdx.y;
  for (long p = blockIdx.x * 256L + threadIdx.x; p < npix; p += (long)gridDim.x * 256) {
    const uint8_t* pa = a + (img * npix + p) * 3;
    const uint8_t* pb = b + (img * npix + p) * 3;
    const float la = (pa[0] / 255.f) * 0.299f + (pa[1] / 255.f) * 0.587f + (pa[2] / 255.f) * 0.114f;
    const float lb = (pb[0] / 255.f) * 0.299f + (pb[1] / 255.f) * 0.587f + (pb[2] / 255.f) * 0.114f;
    ya[img * npix + p] = rintf(la * 255.f);
    yb[img * npix + p] = rintf(lb * 255.f);
  }
}

__global__ __launch_bounds__(256) void avgpool2_kernel(const float* __restrict__ in, int h, int w,
                                                       float* __restrict__ out) {
  const int ho = h / 2, wo = w / 2;
  const long img = blockIdx.y;
  for (long p = blockIdx.x * 256L + threadIdx.x; p < (long)ho * wo; p += (long)gridDim.x * 256) {
    const int oy = (int)(p / wo), ox = (int)(p - (long)oy * wo);
    const float* r0 = in + img * h * w + (long)(2 * oy) * w + 2 * ox;
    out[img * ho * wo + p] = ((r0[0] + r0[1]) + (r0[w] + r0[w + 1])) * 0.25f;
  }
}

// grid (tiles_x, tiles_y, n); partial [n][tiles][2] = (sum ssim, sum cs) over the tile's valid outputs
__global__ __launch_bounds__(256) void ssim_tile_kernel(const float* __restrict__ ya, const float* __restrict__ yb,
                                                        int h, int w, SsimWin win, float c1, float c2,
                                                        float* __restrict__ part) {
  __shared__ float sa[SS_IH][SS_IW], sb[SS_IH][SS_IW];
  __shared__ float hq[5][SS_IH][SS_TW];  // horizontal passes of a, b, a^2, b^2, ab
  __shared__ float red[2][8];
  const int vh = h - 2 * SS_R, vw = w - 2 * SS_R;  // valid output size
  const int x0 = blockIdx.x * SS_TW, y0 = blockIdx.y * SS_TH;
  const long img = blockIdx.z;
  const float* pa = ya + img * h * w;
  const float* pb = yb + img * h * w;
  const int t = threadIdx.x;
  for (int i = t; i < SS_IH * SS_IW; i += 256) {
    const int r = i / SS_IW, c = i - r * SS_IW;
    const int gy = y0 + r, gx = x0 + c;
    const bool in = gy < h && gx < w;
    sa[r][c] = in ? pa[(long)gy * w + gx] : 0.f;
    sb[r][c] = in ? pb[(long)gy * w + gx] : 0.f;
  }
  __syncthreads();
  for (int i = t; i < SS_IH * SS_TW; i += 256) {
    const int r = i / SS_TW, c = i - r * SS_TW;
    float m1 = 0.f, m2 = 0.f, s11 = 0.f, s22 = 0.f, s12 = 0.f;
#pragma unroll
    for (int k = 0; k < SS_W; ++k) {
      const float g = win.g[k], va = sa[r][c + k], vb = sb[r][c + k];
      m1 = fmaf(g, va, m1);
      m2 = fmaf(g, vb, m2);
      s11 = fmaf(g, va * va, s11);
      s22 = fmaf(g, vb * vb, s22);
      s12 = fmaf(g, va * vb, s12);
    }
    hq[0][r][c] = m1; hq[1][r][c] = m2; hq[2][r][c] = s11; hq[3][r][c] = s22; hq[4][r][c] = s12;
  }
  __syncthreads();
  float ss = 0.f, cc = 0.f;
  for (int i = t; i < SS_TH * SS_TW; i += 256) {
    const int r = i / SS_TW, c = i - r * SS_TW;
    if (y0 + r >= vh || x0 + c >= vw) continue;
    float mu1 = 0.f, mu2 = 0.f, e11 = 0.f, e22 = 0.f, e12 = 0.f;
#pragma unroll
    for (int k = 0; k < SS_W; ++k) {
      const float g = win.g[k];
      mu1 = fmaf(g, hq[0][r + k][c], mu1);
      mu2 = fmaf(g, hq[1][r + k][c], mu2);
      e11 = fmaf(g, hq[2][r + k][c], e11);
      e22 = fmaf(g, hq[3][r + k][c], e22);
      e12 = fmaf(g, hq[4][r + k][c], e12);
    }
    const float m11 = mu1 * mu1, m22 = mu2 * mu2, m12 = mu1 * mu2;
    const float sg11 = e11 - m11, sg22 = e22 - m22, sg12 = e12 - m12;
    const float cs = fmaxf((2.f * sg12 + c2) / (sg11 + sg22 + c2), 0.f);
    ss += (2.f * m12 + c1) / (m11 + m22 + c1) * cs;
    cc += cs;
  }
  // fixed-order block reduction: lanes (butterfly), then the 4 waves in order
  ss = warp_sum(ss);
  cc = warp_sum(cc);
  if ((t & 63) == 0) { red[0][t >> 6] = ss; red[1][t >> 6] = cc; }
  __syncthreads();
  if (t == 0) {
    const long tile = (long)blockIdx.y * gridDim.x + blockIdx.x;
    const long ntile = (long)gridDim.x * gridDim.y;
    float* o = part + (img * ntile + tile) * 2;
    o[0] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    o[1] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  }
}

// one block per image: out[img * 2 + {0,1}] = mean ssim, mean cs of the level (fp64 sums)
__global__ __launch_bounds__(256) void ssim_finalize_kernel(const float* __restrict__ part, long ntile, double count,
                                                            float* __restrict__ out, int out_stride) {
  __shared__ double red[2][4];
  const long img = blockIdx.x;
  const int t = threadIdx.x;
  double s = 0.0, c = 0.0;
  for (long i = t; i < ntile; i += 256) {
    s += (double)part[(img * ntile + i) * 2];
    c += (double)part[(img * ntile + i) * 2 + 1];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { s += __shfl_xor(s, o, 64); c += __shfl_xor(c, o, 64); }
  if ((t & 63) == 0) { red[0][t >> 6] = s; red[1][t >> 6] = c; }
  __syncthreads();
  if (t == 0) {
    out[img * out_stride + 0] = (float)(((red[0][0] + red[0][1]) + (red[0][2] + red[0][3])) / count);
    out[img * out_stride + 1] = (float)(((red[1][0] + red[1][1]) + (red[1][2] + red[1][3])) / count);
  }
}

SsimWin gaussian_window() {
  SsimWin w;
  double g[SS_W], sum = 0.0;
  for (int i = 0; i < SS_W; ++i) {
    const double d = i - SS_R;
    g[i] = std::exp(-d * d / (2.0 * 1.5 * 1.5));
    sum += g[i];
  }
  for (int i = 0; i < SS_W; ++i) w.g[i] = (float)(g[i] / sum);
  return w;
}

}  // namespace

extern "C" size_t rdeic_image_ssim_ws_floats(int32_t n, int32_t h, int32_t w, int32_t levels) {
  if (n <= 0 || h <= 0 || w <= 0 || levels <= 0) return 0;
  size_t pyr = 0, parts = 0;
  int hh = h, ww = w;
  for (int l = 0; l < levels; ++l) {
    pyr += (size_t)hh * ww;
    const size_t tiles = (size_t)((ww - 2 * SS_R + SS_TW - 1) / SS_TW) * ((hh - 2 * SS_R + SS_TH - 1) / SS_TH);
    parts = parts > tiles ? parts : tiles;
    hh /= 2;
    ww /= 2;
  }
  return 2 * (size_t)n * pyr + 2 * (size_t)n * parts;
}

extern "C" int rdeic_image_ssim(const uint8_t* a, const uint8_t* b, int32_t n, int32_t h, int32_t w, int32_t levels,
                                float* ws, size_t ws_floats, float* out, void* stream) {
  if (!a || !b || !ws || !out || n <= 0 || levels <= 0 || levels > 8) return RDEIC_EINVAL;
  {  // every level must keep an even size for the 2x2 pooling and a valid 11x11 window
    int hh = h, ww = w;
    for (int l = 0; l < levels; ++l) {
      if (hh < SS_W || ww < SS_W || (l + 1 < levels && (hh % 2 || ww % 2))) return RDEIC_EINVAL;
      hh /= 2;
      ww /= 2;
    }
  }
  if (ws_floats < rdeic_image_ssim_ws_floats(n, h, w, levels)) return RDEIC_ENOSPC;
  hipStream_t s = (hipStream_t)stream;
  const SsimWin win = gaussian_window();
  const float c1 = (0.01f * 255.f) * (0.01f * 255.f), c2 = (0.03f * 255.f) * (0.03f * 255.f);
  // ws: [ya pyramid | yb pyramid] per level (n images each), then the tile partials
  size_t pyr = 0;
  {
    int hh = h, ww = w;
    for (int l = 0; l < levels; ++l) { pyr += (size_t)hh * ww; hh /= 2; ww /= 2; }
  }
  float* ya = ws;
  float* yb = ws + (size_t)n * pyr;
  float* part = ws + 2 * (size_t)n * pyr;
  const long npix = (long)h * w;
  hipLaunchKernelGGL(rgb_to_y_kernel, dim3((unsigned)std::min<long>((npix + 255) / 256, 1024), n), dim3(256), 0, s,
                     a, b, npix, ya, yb);
  int hh = h, ww = w;
  size_t off = 0;
  for (int l = 0; l < levels; ++l) {
    const int vh = hh - 2 * SS_R, vw = ww - 2 * SS_R;
    dim3 grid((vw + SS_TW - 1) / SS_TW, (vh + SS_TH - 1) / SS_TH, n);
    hipLaunchKernelGGL(ssim_tile_kernel, grid, dim3(256), 0, s, ya + (size_t)n * off, yb + (size_t)n * off, hh, ww,
                       win, c1, c2, part);
    hipLaunchKernelGGL(ssim_finalize_kernel, dim3(n), dim3(256), 0, s, part, (long)grid.x * grid.y,
                       (double)vh * vw, out + 2 * l, 2 * levels);
    if (l + 1 < levels) {
      const size_t nxt = off + (size_t)hh * ww;
      const long opix = (long)(hh / 2) * (ww / 2);
      dim3 pg((unsigned)std::min<long>((opix + 255) / 256, 1024), n);
      hipLaunchKernelGGL(avgpool2_kernel, pg, dim3(256), 0, s, ya + (size_t)n * off, hh, ww, ya + (size_t)n * nxt);
      hipLaunchKernelGGL(avgpool2_kernel, pg, dim3(256), 0, s, yb + (size_t)n * off, hh, ww, yb + (size_t)n * nxt);
      off = nxt;
    }
    hh /= 2;
    ww /= 2;
  }
  return launch_status();
}
