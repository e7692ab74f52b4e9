// Image transforms on the device: crop -> Pillow-exact resample (bicubic / bilinear) -> optional
// horizontal flip -> ToTensor (u8 / 255) -> Normalize -> fp16 (or fp32) CHW, for a batch of decoded
// 8-bit RGB images of any sizes.  Replaces the reference's per-image CPU transform workers
// (configs/trainers/MaPLeFederated/*.yaml:8-13 through Dassl's build_transform, torchvision and
// Pillow; trainers/client_datamanager.py:21-103) and the fp16 cast at the model entry
// (trainers/maple.py:336).
//
// Default: ONE launch per batch (aug_fused_kernel, one workgroup per (image, band of output rows),
// taps and the band's uint8 intermediate rows in LDS).  When a batch's taps + band rows would not fit
// 64 KB of LDS (downscale beyond ~6x), three launches instead, all
// byte work (HBM / L2 bound, no MFMA):
//   1. coeff:      one thread per (image, axis, output index) computes Pillow's precompute_coeffs in
//                  float64 with the same operation order (-ffp-contract=off) and the 22-bit
//                  fixed-point taps of normalize_coeffs_8bpc;
//   2. horizontal: one thread per (image, intermediate row, output column): int32 tap sums over the
//                  crop's row -> clip8 -> uint8 intermediate (only rows ybox_first..ybox_last that
//                  the output window reads, as ImagingResampleInner does);
//   3. vertical:   one thread per (image, output row, output column), the vertical taps over the
//                  intermediate, clip8, flip, (u/255 - mean)/std in fp32, stored channel-planar.
// Integer tap sums are exact, so the result is bit-identical to Pillow whatever the summation order.
#include <string.h>

#include "mf_common.h"

namespace {

constexpr int AUG_KMAX = 64;       // taps per output index: downscale factor up to 15.5 (bicubic)
constexpr int AUG_GEOM = 11;       // H, W, y0, x0, ch, cw, RH, RW, oy, ox, flip
constexpr int PRECISION_BITS = 22;  // Pillow Resample.c: 32 - 8 - 2

struct AugDims {
  int B, out_h, out_w, max_rows;
  int64_t coef_off, bound_off, tmp_off;  // byte offsets inside the workspace
};

MF_DEV double aug_filter(double x, int bilinear) {
  if (x < 0.0) x = -x;
  if (bilinear) return x < 1.0 ? 1.0 - x : 0.0;
  const double a = -0.5;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

MF_DEV uint8_t clip8(int v) {
  v >>= PRECISION_BITS;  // arithmetic shift = floor, as Pillow's lookup index
  return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// Pillow precompute_coeffs + normalize_coeffs_8bpc for output index xx of an in_size -> out_size
// resample (box [0, in_size)): writes the fixed-point taps to k[0 .. count) and returns {first, count}
MF_DEV int2 aug_taps(int in_size, int out_size, int xx, int bilinear, int* k, int kcap) {
  const double fsupport = bilinear ? 1.0 : 2.0;
  const double scale = (double)in_size / out_size;
  double filterscale = scale;
  if (filterscale < 1.0) filterscale = 1.0;
  const double support = fsupport * filterscale;
  const double center = 0.0 + (xx + 0.5) * scale;
  const double ss = 1.0 / filterscale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  xmax -= xmin;
  if (xmax > kcap) xmax = kcap;  // unreachable: the host checks the tap count
  double w[AUG_KMAX];
  double ww = 0.0;
  for (int x = 0; x < xmax; ++x) {
    w[x] = aug_filter((x + xmin - center + 0.5) * ss, bilinear);
    ww += w[x];
  }
  for (int x = 0; x < xmax; ++x) {
    const double kx = ww != 0.0 ? w[x] / ww : w[x];
    k[x] = kx < 0 ? (int)(-0.5 + kx * (1 << PRECISION_BITS)) : (int)(0.5 + kx * (1 << PRECISION_BITS));
  }
  return make_int2(xmin, xmax);
}

// coefficient tables: ws coef [B][2][OUT][KMAX] int32, bounds [B][2][OUT] int2 {first, count};
// axis 0 = rows (in = crop height ch, out = RH, window oy), axis 1 = columns (cw, RW, ox)
__global__ __launch_bounds__(256) void aug_coeff_kernel(const int* __restrict__ geom, AugDims d, int bilinear,
                                                        uint8_t* __restrict__ ws) {
  const int OUT = d.out_h > d.out_w ? d.out_h : d.out_w;
  const int j = blockIdx.x * 256 + threadIdx.x;
  const int axis = blockIdx.y, b = blockIdx.z;
  const int* g = geom + b * AUG_GEOM;
  const int n_out = axis ? d.out_w : d.out_h;
  if (j >= n_out) return;
  int* k = (int*)(ws + d.coef_off) + (((int64_t)b * 2 + axis) * OUT + j) * AUG_KMAX;
  const int2 bd = aug_taps(axis ? g[5] : g[4], axis ? g[7] : g[6], j + (axis ? g[9] : g[8]), bilinear, k, AUG_KMAX);
  *((int2*)(ws + d.bound_off) + ((int64_t)b * 2 + axis) * OUT + j) = bd;
}

// horizontal pass: tmp[b][r][x][c] for r in [0, ybox_last - ybox_first)
__global__ __launch_bounds__(256) void aug_horizontal_kernel(const uint8_t* __restrict__ src,
                                                             const int64_t* __restrict__ src_off,
                                                             const int* __restrict__ geom, AugDims d,
                                                             uint8_t* __restrict__ ws) {
  const int OUT = d.out_h > d.out_w ? d.out_h : d.out_w;
  const int x = blockIdx.x * 64 + (threadIdx.x & 63);
  const int r = blockIdx.y * 4 + (threadIdx.x >> 6);
  const int b = blockIdx.z;
  if (x >= d.out_w) return;
  const int* g = geom + b * AUG_GEOM;
  const int2* vb = (const int2*)(ws + d.bound_off) + ((int64_t)b * 2 + 0) * OUT;
  const int y_first = vb[0].x;
  const int y_last = vb[d.out_h - 1].x + vb[d.out_h - 1].y;
  if (r >= y_last - y_first) return;
  const int2 hb = ((const int2*)(ws + d.bound_off))[((int64_t)b * 2 + 1) * OUT + x];
  const int* k = (const int*)(ws + d.coef_off) + (((int64_t)b * 2 + 1) * OUT + x) * AUG_KMAX;
  const int W = g[1];
  const uint8_t* row = src + src_off[b] + ((int64_t)(g[2] + y_first + r) * W + g[3] + hb.x) * 3;
  int s0 = 1 << (PRECISION_BITS - 1), s1 = s0, s2 = s0;
  for (int t = 0; t < hb.y; ++t) {
    const int kt = k[t];
    s0 += (int)row[3 * t + 0] * kt;
    s1 += (int)row[3 * t + 1] * kt;
    s2 += (int)row[3 * t + 2] * kt;
  }
  uint8_t* o = ws + d.tmp_off + (((int64_t)b * d.max_rows + r) * d.out_w + x) * 3;
  o[0] = clip8(s0);
  o[1] = clip8(s1);
  o[2] = clip8(s2);
}

// vertical pass + flip + ToTensor + Normalize, channel-planar out [b][3][out_h][out_w]
template <bool F16>
__global__ __launch_bounds__(256) void aug_vertical_kernel(const int* __restrict__ geom, AugDims d,
                                                           const uint8_t* __restrict__ ws, float m0, float m1,
                                                           float m2, float sd0, float sd1, float sd2,
                                                           void* __restrict__ out) {
  const int OUT = d.out_h > d.out_w ? d.out_h : d.out_w;
  const int x = blockIdx.x * 64 + (threadIdx.x & 63);
  const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
  const int b = blockIdx.z;
  if (x >= d.out_w || y >= d.out_h) return;
  const int* g = geom + b * AUG_GEOM;
  const int2* vb = (const int2*)(ws + d.bound_off) + ((int64_t)b * 2 + 0) * OUT;
  const int y_first = vb[0].x;
  const int2 bd = vb[y];
  const int* k = (const int*)(ws + d.coef_off) + (((int64_t)b * 2 + 0) * OUT + y) * AUG_KMAX;
  const int xs = g[10] ? d.out_w - 1 - x : x;  // RandomHorizontalFlip after the resize
  const uint8_t* col = ws + d.tmp_off + (((int64_t)b * d.max_rows + (bd.x - y_first)) * d.out_w + xs) * 3;
  const int64_t rstride = (int64_t)d.out_w * 3;
  int s0 = 1 << (PRECISION_BITS - 1), s1 = s0, s2 = s0;
  for (int t = 0; t < bd.y; ++t) {
    const int kt = k[t];
    s0 += (int)col[t * rstride + 0] * kt;
    s1 += (int)col[t * rstride + 1] * kt;
    s2 += (int)col[t * rstride + 2] * kt;
  }
  // torchvision ToTensor: float(u) / 255; Normalize: (v - mean) / std, each correctly rounded in fp32
  const float v0 = ((float)clip8(s0) / 255.0f - m0) / sd0;
  const float v1 = ((float)clip8(s1) / 255.0f - m1) / sd1;
  const float v2 = ((float)clip8(s2) / 255.0f - m2) / sd2;
  const int64_t plane = (int64_t)d.out_h * d.out_w;
  const int64_t o = (int64_t)b * 3 * plane + (int64_t)y * d.out_w + x;
  if (F16) {
    f16* p = (f16*)out;
    p[o] = (f16)v0;
    p[o + plane] = (f16)v1;
    p[o + 2 * plane] = (f16)v2;
  } else {
    float* p = (float*)out;
    p[o] = v0;
    p[o + plane] = v1;
    p[o + 2 * plane] = v2;
  }
}

// Fused path: one workgroup per (image, band of `band` output rows).  The horizontal taps of the
// window's columns, the band's vertical taps and the uint8 intermediate rows the band reads all sit
// in LDS (dynamic: out_w*kh + band*kv ints, out_w + band int2, rows_max*out_w*3 bytes), so the
// intermediate never goes to HBM and the batch is one launch.  Same integer arithmetic as the
// three-launch path: bit-identical output.
constexpr int AUG_ARG_IMAGES = 64;  // images per fused launch: their geometry rides in the kernel arguments
struct AugBatchArg {
  int64_t off[AUG_ARG_IMAGES];
  int geom[AUG_ARG_IMAGES * AUG_GEOM];
};  // 3 328 bytes (< the 4 KB kernel-argument segment): no host->device copy before the launch

template <bool F16>
__global__ __launch_bounds__(256) void aug_fused_kernel(const uint8_t* __restrict__ src, const AugBatchArg ba,
                                                        int b_base, int out_h, int out_w,
                                                        int bilinear, int band, int kh, int kv, int rows_max,
                                                        float m0, float m1, float m2, float sd0,
                                                        float sd1, float sd2, void* __restrict__ out) {
  extern __shared__ int aug_lds[];
  int* hk = aug_lds;                         // [out_w][kh]
  int* vk = hk + out_w * kh;                 // [band][kv]
  int2* hb = (int2*)(vk + band * kv);        // [out_w]   (8-byte aligned: the int counts are even)
  int2* vbd = hb + out_w;                    // [band]
  uint8_t* tmp = (uint8_t*)(vbd + band);     // [rows_max][out_w][3]
  const int bl = blockIdx.y, b = b_base + bl;
  const int y0 = blockIdx.x * band;
  const int nrows = out_h - y0 < band ? out_h - y0 : band;
  const int* g = ba.geom + bl * AUG_GEOM;
  for (int j = threadIdx.x; j < out_w + nrows; j += 256) {
    if (j < out_w) hb[j] = aug_taps(g[5], g[7], g[9] + j, bilinear, hk + j * kh, kh);
    else vbd[j - out_w] = aug_taps(g[4], g[6], g[8] + y0 + (j - out_w), bilinear, vk + (j - out_w) * kv, kv);
  }
  __syncthreads();
  const int y_first = vbd[0].x;
  int nr = vbd[nrows - 1].x + vbd[nrows - 1].y - y_first;
  if (nr > rows_max) nr = rows_max;  // unreachable: the host sizes rows_max from the band's span
  const int W = g[1];
  const uint8_t* img = src + ba.off[bl] + ((int64_t)(g[2] + y_first) * W + g[3]) * 3;
  for (int e = threadIdx.x; e < nr * out_w; e += 256) {
    const int r = e / out_w, x = e - r * out_w;
    const int2 bd = hb[x];
    const int* k = hk + x * kh;
    const uint8_t* row = img + ((int64_t)r * W + bd.x) * 3;
    int s0 = 1 << (PRECISION_BITS - 1), s1 = s0, s2 = s0;
    for (int t = 0; t < bd.y; ++t) {
      const int kt = k[t];
      s0 += (int)row[3 * t + 0] * kt;
      s1 += (int)row[3 * t + 1] * kt;
      s2 += (int)row[3 * t + 2] * kt;
    }
    uint8_t* o = tmp + (r * out_w + x) * 3;
    o[0] = clip8(s0);
    o[1] = clip8(s1);
    o[2] = clip8(s2);
  }
  __syncthreads();
  const int64_t plane = (int64_t)out_h * out_w;
  const int flip = g[10];
  for (int e = threadIdx.x; e < nrows * out_w; e += 256) {
    const int yl = e / out_w, x = e - yl * out_w;
    const int2 bd = vbd[yl];
    const int* k = vk + yl * kv;
    const int xs = flip ? out_w - 1 - x : x;
    int r0 = bd.x - y_first;
    int n = bd.y;
    if (r0 + n > nr) n = nr - r0;
    const uint8_t* col = tmp + (r0 * out_w + xs) * 3;
    int s0 = 1 << (PRECISION_BITS - 1), s1 = s0, s2 = s0;
    for (int t = 0; t < n; ++t) {
      const int kt = k[t];
      s0 += (int)col[t * out_w * 3 + 0] * kt;
      s1 += (int)col[t * out_w * 3 + 1] * kt;
      s2 += (int)col[t * out_w * 3 + 2] * kt;
    }
    const float v0 = ((float)clip8(s0) / 255.0f - m0) / sd0;
    const float v1 = ((float)clip8(s1) / 255.0f - m1) / sd1;
    const float v2 = ((float)clip8(s2) / 255.0f - m2) / sd2;
    const int64_t o = (int64_t)b * 3 * plane + (int64_t)(y0 + yl) * out_w + x;
    if (F16) {
      f16* p = (f16*)out;
      p[o] = (f16)v0;
      p[o + plane] = (f16)v1;
      p[o + 2 * plane] = (f16)v2;
    } else {
      float* p = (float*)out;
      p[o] = v0;
      p[o + plane] = v1;
      p[o + 2 * plane] = v2;
    }
  }
}

constexpr int64_t AUG_FUSED_LDS_MAX = 64 * 1024;

int64_t aug_fused_lds(int out_w, int band, int kh, int kv, int rows_max) {
  return ((int64_t)out_w * kh + (int64_t)band * kv) * 4 + ((int64_t)out_w + band) * 8 + (int64_t)rows_max * out_w * 3;
}

AugDims aug_dims(int B, int out_h, int out_w, int max_rows) {
  const int OUT = out_h > out_w ? out_h : out_w;
  AugDims d{B, out_h, out_w, max_rows, 0, 0, 0};
  d.coef_off = ((int64_t)B * AUG_GEOM * sizeof(int) + 255) / 256 * 256;  // geometry copy lives in front
  d.bound_off = d.coef_off + (int64_t)B * 2 * OUT * AUG_KMAX * sizeof(int);
  d.tmp_off = d.bound_off + (int64_t)B * 2 * OUT * 8;
  d.tmp_off = (d.tmp_off + 255) / 256 * 256;
  return d;
}

int64_t aug_ws_bytes(const AugDims& d) {
  return d.tmp_off + (int64_t)d.B * d.max_rows * d.out_w * 3;
}

}  // namespace

extern "C" int64_t mf_augment_ws_bytes(int B, int out_h, int out_w, int max_rows) {
  if (B <= 0 || out_h <= 0 || out_w <= 0 || max_rows <= 0) return -1;
  return aug_ws_bytes(aug_dims(B, out_h, out_w, max_rows));
}

// geom_host: B x 11 int32 {H, W, y0, x0, ch, cw, RH, RW, oy, ox, flip} (host memory, validated here);
// src_off: device int64 [B] byte offsets of each HWC uint8 image inside src (src_bytes long).
extern "C" int mf_augment(const void* src, int64_t src_bytes, const int64_t* src_off_host, const int64_t* src_off,
                          const int* geom_host, int B, int out_h, int out_w, int interp, float m0, float m1,
                          float m2, float s0, float s1, float s2, void* out, int out_f16, void* ws,
                          int64_t ws_bytes, void* stream) {
  if (B <= 0) return 0;
  if (out_h <= 0 || out_w <= 0 || out_h > 4096 || out_w > 4096)
    return mf_set_error("mf_augment: output size must be in 1..4096", -1);
  if (interp != 0 && interp != 1) return mf_set_error("mf_augment: interp is 0 (bicubic) or 1 (bilinear)", -1);
  if (!src || !src_off_host || !src_off || !geom_host || !out || !ws)
    return mf_set_error("mf_augment: null pointer", -1);
  int max_rows = 1, kh = 1, kv = 1;
  double vscale = 1.0, vsupport = 0.0;  // the largest vertical scale / support over the batch
  const double fsup = interp == 1 ? 1.0 : 2.0;
  for (int b = 0; b < B; ++b) {
    const int* g = geom_host + b * AUG_GEOM;
    const int H = g[0], W = g[1], y0 = g[2], x0 = g[3], ch = g[4], cw = g[5], RH = g[6], RW = g[7], oy = g[8],
              ox = g[9];
    if (H <= 0 || W <= 0 || ch <= 0 || cw <= 0 || y0 < 0 || x0 < 0 || y0 + ch > H || x0 + cw > W)
      return mf_set_error("mf_augment: crop box outside the image", -1);
    if (RH <= 0 || RW <= 0 || oy < 0 || ox < 0 || oy + out_h > RH || ox + out_w > RW)
      return mf_set_error("mf_augment: output window outside the resized image", -1);
    if (src_off_host[b] < 0 || src_off_host[b] + (int64_t)H * W * 3 > src_bytes)
      return mf_set_error("mf_augment: image extends past the source buffer", -1);
    for (int axis = 0; axis < 2; ++axis) {
      const double sc = (double)(axis ? cw : ch) / (axis ? RW : RH);
      const double fs = sc < 1.0 ? 1.0 : sc;
      const int taps = (int)ceil(fsup * fs) * 2 + 1;
      if (taps > AUG_KMAX) return mf_set_error("mf_augment: downscale factor too large (taps > 64)", -1);
      if (axis) kh = taps > kh ? taps : kh;
      else {
        kv = taps > kv ? taps : kv;
        vscale = sc > vscale ? sc : vscale;
        vsupport = fsup * fs > vsupport ? fsup * fs : vsupport;
      }
    }
    if (ch > max_rows) max_rows = ch;
  }
  const AugDims d = aug_dims(B, out_h, out_w, max_rows);
  if (aug_ws_bytes(d) > ws_bytes) return mf_set_error("mf_augment: workspace too small", -1);
  hipStream_t st = (hipStream_t)stream;
  // fused path: the largest band (16 rows down to 1) whose taps + intermediate rows fit 64 KB of LDS;
  // a band of n output rows reads at most (n-1)*scale + 2*support + 2 intermediate rows.  Geometry and
  // offsets travel by value in the kernel arguments, 64 images per launch.
  {
    for (int band = 16; band >= 1; band /= 2) {
      int rows = (int)ceil((band - 1) * vscale + 2.0 * vsupport) + 3;
      if (rows > max_rows) rows = max_rows;
      const int kh2 = (kh + 1) & ~1, kv2 = (kv + 1) & ~1;  // even counts keep the int2 arrays aligned
      int64_t lds = aug_fused_lds(out_w, band, kh2, kv2, rows);
      if (lds > AUG_FUSED_LDS_MAX) continue;
      for (int b0 = 0; b0 < B; b0 += AUG_ARG_IMAGES) {
        const int nb = B - b0 < AUG_ARG_IMAGES ? B - b0 : AUG_ARG_IMAGES;
        AugBatchArg ba;
        memset(&ba, 0, sizeof(ba));
        memcpy(ba.off, src_off_host + b0, (size_t)nb * sizeof(int64_t));
        memcpy(ba.geom, geom_host + (size_t)b0 * AUG_GEOM, (size_t)nb * AUG_GEOM * sizeof(int));
        const dim3 gf((out_h + band - 1) / band, nb);
        if (out_f16)
          aug_fused_kernel<true><<<gf, 256, lds, st>>>((const uint8_t*)src, ba, b0, out_h, out_w, interp, band, kh2,
                                                       kv2, rows, m0, m1, m2, s0, s1, s2, out);
        else
          aug_fused_kernel<false><<<gf, 256, lds, st>>>((const uint8_t*)src, ba, b0, out_h, out_w, interp, band, kh2,
                                                        kv2, rows, m0, m1, m2, s0, s1, s2, out);
        MF_CHECK_LAUNCH();
      }
      return 0;
    }
  }
  int* geom_dev = (int*)ws;  // the geometry travels in the workspace's first bytes
  if (hipMemcpyAsync(geom_dev, geom_host, (size_t)B * AUG_GEOM * sizeof(int), hipMemcpyHostToDevice, st) !=
      hipSuccess)
    return mf_set_error("mf_augment: geometry upload failed", -1);
  const int OUT = out_h > out_w ? out_h : out_w;
  aug_coeff_kernel<<<dim3((OUT + 255) / 256, 2, B), 256, 0, st>>>(geom_dev, d, interp, (uint8_t*)ws);
  MF_CHECK_LAUNCH();
  aug_horizontal_kernel<<<dim3((out_w + 63) / 64, (max_rows + 3) / 4, B), 256, 0, st>>>(
      (const uint8_t*)src, src_off, geom_dev, d, (uint8_t*)ws);
  MF_CHECK_LAUNCH();
  const dim3 gv((out_w + 63) / 64, (out_h + 3) / 4, B);
  if (out_f16)
    aug_vertical_kernel<true><<<gv, 256, 0, st>>>(geom_dev, d, (const uint8_t*)ws, m0, m1, m2, s0, s1, s2, out);
  else
    aug_vertical_kernel<false><<<gv, 256, 0, st>>>(geom_dev, d, (const uint8_t*)ws, m0, m1, m2, s0, s1, s2, out);
  MF_CHECK_LAUNCH();
  return 0;
}
