// ImageViT input transforms on device: the reference's torchvision
// pipelines on PIL images, `data/image_dataset.py:139-173`:
//   train: Resize((S,S)) -> RandomHorizontalFlip(0.5) -> RandomRotation(15) ->
//          ColorJitter(0.2, 0.2, 0.2, 0.1) -> RandomAffine(0, translate (0.1,0.1), scale (0.9,1.1))
//          -> ToTensor -> Normalize(ImageNet)
//   val  : Resize((S,S)) -> ToTensor -> Normalize
// One workgroup per image, output fp32 NCHW [B][3][S][S] (the patch-embed im2col input).
//
// Emulated PIL arithmetic (what torchvision runs for PIL images):
//  * Resize BILINEAR = PIL's separable resampler: triangle filter with support scaled by
//    max(in/out, 1) (antialiasing when shrinking), coefficients in 22-bit fixed point, a
//    horizontal pass rounded and clipped to uint8, then the vertical pass (ImagingResample);
//  * rotate / affine NEAREST = PIL's affine transform: source = M * (x + 0.5, y + 0.5),
//    truncated to the pixel, outside -> fill 0; M built as Image.rotate and torchvision's
//    _get_inverse_affine_matrix build it;
//  * ColorJitter = ImageEnhance Brightness / Contrast / Color (Image.blend: in1 + a*(in2-in1),
//    truncated and clipped to uint8; grayscale L = (19595 R + 38470 G + 7471 B + 2^15) >> 16;
//    contrast mean = round(mean L)) and hue (PIL's 8-bit HSV round trip) in a random order,
//    each step stored as uint8 like a PIL image; ToTensor / Normalize in fp32 as torch does.
// Random parameters come from fer_image_aug_draw (counter hash, one record per image), so a
// test can also pass explicit ones. The contrast mean needs the whole jittered image, hence
// two passes over the pixels (the second recomputes the geometry: a bilinear tap set is cheap).
#include "common.h"
#include "fervit_internal.h"

// PIL's x86-64 build evaluates a*b+c as two rounded operations; hipcc contracts to FMA by
// default, which moves truncated blends / fixed-point coordinates by one step.
#pragma clang fp contract(off)

namespace fer {

constexpr int IMG_NP = 16;  // floats per image parameter record
// record: [0] flip, [1] angle (deg), [2] brightness f, [3] contrast f, [4] saturation f,
//         [5] hue f, [6..9] jitter order (op ids 0..3 = b, c, s, h), [10] tx, [11] ty, [12] scale,
//         [13] hue enabled (torchvision skips the HSV round trip when ColorJitter's hue is 0)

struct ImgSrc {
  const uint8_t* p;
  int H, W, C;
};

// PIL bilinear resample taps for output index o (in -> out): window [lo, lo+n) and the weight
// normaliser; weight i in 22-bit fixed point is tap_k(). No tap-count limit (antialiased
// shrinking widens the window), weights recomputed rather than stored (no scratch).
struct Taps {
  int lo, n;
  double center, ss, tot;
};
FER_DEV void pil_taps(int o, int in, int out, Taps& t) {
  const double scale = (double)in / out;
  const double fs = scale > 1.0 ? scale : 1.0;
  const double support = 1.0 * fs;
  t.center = (o + 0.5) * scale;
  t.ss = 1.0 / fs;
  int xmin = (int)(t.center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(t.center + support + 0.5);
  if (xmax > in) xmax = in;
  t.lo = xmin;
  t.n = xmax - xmin;
  t.tot = 0.0;
  for (int i = 0; i < t.n; ++i) {
    double x = (i + xmin - t.center + 0.5) * t.ss;
    if (x < 0) x = -x;
    t.tot += x < 1.0 ? 1.0 - x : 0.0;
  }
}
FER_DEV int tap_k(const Taps& t, int i) {
  double x = (i + t.lo - t.center + 0.5) * t.ss;
  if (x < 0) x = -x;
  const double w = x < 1.0 ? 1.0 - x : 0.0;
  const double v = t.tot != 0.0 ? w / t.tot : 0.0;
  return (int)(v < 0 ? -0.5 + v * (1 << 22) : 0.5 + v * (1 << 22));
}
FER_DEV int clip8(long v) { return v < 0 ? 0 : (v > 255 ? 255 : (int)v); }

// resized (S x S, uint8 RGB) pixel (x, y) of the source
FER_DEV void resized_px(const ImgSrc& s, int S, int x, int y, int rgb[3]) {
  Taps tx, ty;
  pil_taps(x, s.W, S, tx);
  pil_taps(y, s.H, S, ty);
  long acc[3] = {1L << 21, 1L << 21, 1L << 21};
  for (int j = 0; j < ty.n; ++j) {
    const uint8_t* row = s.p + (long)(ty.lo + j) * s.W * s.C;
    long h[3] = {1L << 21, 1L << 21, 1L << 21};
    for (int i = 0; i < tx.n; ++i) {
      const uint8_t* px = row + (long)(tx.lo + i) * s.C;
      const long k = tap_k(tx, i);
      if (s.C == 1) {
        h[0] += (long)px[0] * k;
      } else {
        h[0] += (long)px[0] * k;
        h[1] += (long)px[1] * k;
        h[2] += (long)px[2] * k;
      }
    }
    if (s.C == 1) h[1] = h[2] = h[0];
    const long ky = tap_k(ty, j);
    for (int c = 0; c < 3; ++c) acc[c] += (long)clip8(h[c] >> 22) * ky;
  }
  for (int c = 0; c < 3; ++c) rgb[c] = clip8(acc[c] >> 22);
}

FER_DEV int pil_L(const int rgb[3]) { return (rgb[0] * 19595 + rgb[1] * 38470 + rgb[2] * 7471 + 0x8000) >> 16; }
FER_DEV int blend8(int a, int b, float alpha) {  // Image.blend(im1=a, im2=b, alpha)
  const float t = ((float)a + (alpha * (float)(b - a)));
  return t <= 0.f ? 0 : (t >= 255.f ? 255 : (int)t);
}

// torchvision adjust_hue on a PIL image: RGB -> HSV (PIL's 8-bit conversion), h += uint8(hf*255)
// (wrapping), HSV -> RGB. The float/double mix is PIL's (Convert.c rgb2hsv_row / hsv2rgb, whose
// float temporaries round where the C code stores into a float); checked against PIL over all
// 2^24 inputs of each direction (tests/golden/make_image_golden.py).
FER_DEV void hue_shift(int rgb[3], float hf) {
  const int r = rgb[0], g = rgb[1], b = rgb[2];
  const int mx = max(r, max(g, b)), mn = min(r, min(g, b));
  if (mx == mn) return;  // s = 0: hue moves nothing, v = r = g = b
  const float cr = (float)(mx - mn);
  const float s = cr / (float)mx;
  const float rc = (float)(mx - r) / cr, gc = (float)(mx - g) / cr, bc = (float)(mx - b) / cr;
  float h;
  if (r == mx) h = bc - gc;
  else if (g == mx) h = (float)((2.0 + (double)rc) - (double)bc);
  else h = (float)((4.0 + (double)gc) - (double)rc);
  h = (float)fmod((double)h / 6.0 + 1.0, 1.0);
  int uh = clip8((long)(((double)h * 255.0)));
  const int us = clip8((long)(((double)s * 255.0)));
  const int v = mx;
  uh = (uh + (((int)((double)hf * 255.0)) & 255)) & 255;
  if (us == 0) {
    rgb[0] = rgb[1] = rgb[2] = v;
    return;
  }
  const double hd = (double)uh * 6.0 / 255.0;
  const int i = (int)floor(hd);
  const float f = (float)(hd - (double)i);
  const float fs = (float)((double)us / 255.0);
  const double vd = (double)v;
  const int p = clip8((long)round(vd * (1.0 - (double)fs)));
  const int q = clip8((long)round(vd * (1.0 - (double)(fs * f))));
  const int t = clip8((long)round(vd * (1.0 - (double)fs * (1.0 - (double)f))));
  switch (i % 6) {
    case 0: rgb[0] = v; rgb[1] = t; rgb[2] = p; break;
    case 1: rgb[0] = q; rgb[1] = v; rgb[2] = p; break;
    case 2: rgb[0] = p; rgb[1] = v; rgb[2] = t; break;
    case 3: rgb[0] = p; rgb[1] = q; rgb[2] = v; break;
    case 4: rgb[0] = t; rgb[1] = p; rgb[2] = v; break;
    default: rgb[0] = v; rgb[1] = p; rgb[2] = q; break;
  }
}

// one jitter op on a uint8 RGB pixel; contrast uses the image mean (round(mean L))
FER_DEV void jitter_op(int op, int rgb[3], const float* P, int cmean) {
  if (op == 0) {
    for (int c = 0; c < 3; ++c) rgb[c] = blend8(0, rgb[c], P[2]);
  } else if (op == 1) {
    for (int c = 0; c < 3; ++c) rgb[c] = blend8(cmean, rgb[c], P[3]);
  } else if (op == 2) {
    const int l = pil_L(rgb);
    for (int c = 0; c < 3; ++c) rgb[c] = blend8(l, rgb[c], P[4]);
  } else if (P[13] != 0.f) {  // hue enabled (ColorJitter hue > 0): HSV round trip even at 0
    hue_shift(rgb, P[5]);
  }
}

// Per-image geometry, built once per workgroup in LDS with PIL's own double arithmetic:
//  rotation: Image.rotate's matrix, then ImagingTransformAffine's 16.16 fixed-point path
//            (affine_fixed): src = (a2 + x*a0 + y*a1) >> 16, (a5 + x*a3 + y*a4) >> 16;
//  affine  : torchvision's _get_inverse_affine_matrix (angle 0, no shear) is a pure scale +
//            translation, so PIL takes ImagingScaleAffine: per-axis tables from the running
//            double sums xo += a0 (COORD: negative -> -1 = outside).
FER_DEV void rotation_fixed(float angle_deg, int S, int r[6]) {
  double ang = (double)angle_deg;
  ang = ang - 360.0 * floor(ang / 360.0);  // Python's angle % 360.0
  const double th = -(ang * (3.141592653589793 / 180.0));
  const double cs = nearbyint(cos(th) * 1e15) / 1e15, sn = nearbyint(sin(th) * 1e15) / 1e15;
  const double a = cs, b = sn, d = -sn, e = cs, cx = S / 2.0, cy = S / 2.0;
  double c = (((a * -cx) + (b * -cy)) + 0.0) + cx;
  double f = (((d * -cx) + (e * -cy)) + 0.0) + cy;
  auto fix = [](double v) {
    const double t = v * 65536.0 + 0.5;
    return t < 0.0 ? (int)floor(t) : (int)t;
  };
  r[0] = fix(a);
  r[1] = fix(b);
  r[3] = fix(d);
  r[4] = fix(e);
  r[2] = fix(((c + a * 0.5) + b * 0.5));
  r[5] = fix(((f + d * 0.5) + e * 0.5));
}

// pixel (x, y) of the rotated, flipped, resized image (before ColorJitter); fill 0 outside
FER_DEV void rotated_px(const ImgSrc& s, int S, bool flip, const int* r, int x, int y, int rgb[3]) {
  const int xin = (r[2] + x * r[0] + y * r[1]) >> 16, yin = (r[5] + x * r[3] + y * r[4]) >> 16;
  if (xin < 0 || yin < 0 || xin >= S || yin >= S) {
    rgb[0] = rgb[1] = rgb[2] = 0;
    return;
  }
  resized_px(s, S, flip ? S - 1 - xin : xin, yin, rgb);
}

constexpr int IMG_MAXS = 1024;

__global__ __launch_bounds__(256) void image_augment_kernel(const uint8_t* __restrict__ src,
                                                            const int64_t* __restrict__ off,
                                                            const int32_t* __restrict__ hwc, int S,
                                                            float* __restrict__ out, const float* __restrict__ prm,
                                                            int train, float m0, float m1, float m2, float s0, float s1,
                                                            float s2) {
  __shared__ float P[IMG_NP];
  __shared__ int R[6];
  __shared__ int xtab[IMG_MAXS], ytab[IMG_MAXS];
  __shared__ long red[4];
  const int b = blockIdx.x, tid = threadIdx.x;
  if (tid < IMG_NP) P[tid] = train ? prm[(long)b * IMG_NP + tid] : 0.f;
  const ImgSrc s{src + off[b], hwc[3 * b], hwc[3 * b + 1], hwc[3 * b + 2]};
  __syncthreads();
  const int npx = S * S;
  const float mean[3] = {m0, m1, m2}, sd[3] = {s0, s1, s2};
  float* o = out + (long)b * 3 * npx;
  if (!train) {
    for (int p = tid; p < npx; p += 256) {
      int rgb[3];
      resized_px(s, S, p % S, p / S, rgb);
      for (int c = 0; c < 3; ++c) o[(long)c * npx + p] = ((float)rgb[c] / 255.f - mean[c]) / sd[c];
    }
    return;
  }
  if (tid == 0) rotation_fixed(P[1], S, R);
  {
    // RandomAffine inverse matrix (torchvision, PIL branch): a0 = a4 = 1/scale,
    // a2 = (1/scale)(-c - tx) + c, a5 likewise, c = S * 0.5
    const double inv = 1.0 / (double)P[12], cx = S * 0.5;
    const double a2 = (0.0 + (inv * (-cx - (double)P[10]) + 0.0 * (-cx - (double)P[11]))) + cx;
    const double a5 = (0.0 + (-0.0 * (-cx - (double)P[10]) + inv * (-cx - (double)P[11]))) + cx;
    for (int t = tid; t < 2 * S; t += 256) {
      const int i = t < S ? t : t - S;
      double v = (t < S ? a2 : a5) + inv * 0.5;
      for (int k = 0; k < i; ++k) v += inv;
      const int c = v < 0.0 ? -1 : (int)v;
      (t < S ? xtab : ytab)[i] = c < S ? c : -1;
    }
  }
  __syncthreads();
  int r[6];
  for (int k = 0; k < 6; ++k) r[k] = R[k];
  const bool flip = P[0] != 0.f;
  int ord[4];
  for (int k = 0; k < 4; ++k) ord[k] = (int)P[6 + k];
  int cpos = 0;
  while (cpos < 4 && ord[cpos] != 1) ++cpos;
  // pass 1: mean L of the image the contrast op sees (ops before it applied)
  long sum = 0;
  for (int p = tid; p < npx; p += 256) {
    int rgb[3];
    rotated_px(s, S, flip, r, p % S, p / S, rgb);
    for (int k = 0; k < cpos; ++k) jitter_op(ord[k], rgb, P, 0);
    sum += pil_L(rgb);
  }
  for (int d = 32; d > 0; d >>= 1) sum += __shfl_xor(sum, d, 64);
  if ((tid & 63) == 0) red[tid >> 6] = sum;
  __syncthreads();
  const int cmean = (int)((double)(red[0] + red[1] + red[2] + red[3]) / npx + 0.5);
  // pass 2: RandomAffine (nearest, fill 0 AFTER the jitter) of the jittered image
  for (int p = tid; p < npx; p += 256) {
    const int xi = xtab[p % S], yi = ytab[p / S];
    int rgb[3] = {0, 0, 0};
    if (xi >= 0 && yi >= 0) {
      rotated_px(s, S, flip, r, xi, yi, rgb);
      for (int k = 0; k < 4; ++k) jitter_op(ord[k], rgb, P, cmean);
    }
    for (int c = 0; c < 3; ++c) o[(long)c * npx + p] = ((float)rgb[c] / 255.f - mean[c]) / sd[c];
  }
}

// per-image random parameters (torchvision's get_params ranges), counter-hash draws
FER_DEV float hu(uint64_t seed, uint32_t k) { return ((float)(fer_hash(seed, k) >> 8) + 0.5f) * (1.f / 16777216.f); }
__global__ void image_aug_draw_kernel(float* __restrict__ prm, int B, int S, fer_image_aug a, uint64_t seed) {
  seed = step_seed(seed);
  const int b = blockIdx.x * 64 + threadIdx.x;
  if (b >= B) return;
  float* P = prm + (long)b * IMG_NP;
  const uint32_t k = (uint32_t)b * 16u;
  P[0] = hu(seed, k) < a.flip_p ? 1.f : 0.f;
  P[1] = -a.degrees + 2.f * a.degrees * hu(seed, k + 1);
  P[2] = fmaxf(0.f, 1.f - a.brightness) + (1.f + a.brightness - fmaxf(0.f, 1.f - a.brightness)) * hu(seed, k + 2);
  P[3] = fmaxf(0.f, 1.f - a.contrast) + (1.f + a.contrast - fmaxf(0.f, 1.f - a.contrast)) * hu(seed, k + 3);
  P[4] = fmaxf(0.f, 1.f - a.saturation) + (1.f + a.saturation - fmaxf(0.f, 1.f - a.saturation)) * hu(seed, k + 4);
  P[5] = -a.hue + 2.f * a.hue * hu(seed, k + 5);
  int ord[4] = {0, 1, 2, 3};  // torch.randperm(4) -> Fisher-Yates
  for (int i = 3; i > 0; --i) {
    const int j = (int)(hu(seed, k + 6 + i) * (i + 1)) % (i + 1);
    const int t = ord[i];
    ord[i] = ord[j];
    ord[j] = t;
  }
  for (int i = 0; i < 4; ++i) P[6 + i] = (float)ord[i];
  const float mdx = a.translate * S;
  P[10] = rintf(-mdx + 2.f * mdx * hu(seed, k + 10));
  P[11] = rintf(-mdx + 2.f * mdx * hu(seed, k + 11));
  P[12] = a.scale_lo + (a.scale_hi - a.scale_lo) * hu(seed, k + 12);
  P[13] = a.hue > 0.f ? 1.f : 0.f;
  P[14] = P[15] = 0.f;
}

}  // namespace fer

using namespace fer;

extern "C" int fer_image_aug_draw(float* params, int B, int S, const fer_image_aug* aug, uint64_t seed,
                                  fer_stream_t stream) {
  if (B <= 0) return 0;
  if (!aug || !params) return set_error("image_aug_draw: null argument");
  hipLaunchKernelGGL(image_aug_draw_kernel, dim3(ceil_div(B, 64)), dim3(64), 0, (hipStream_t)stream, params, B, S,
                     *aug, seed);
  return hip_check("image_aug_draw");
}

extern "C" int fer_image_augment(const uint8_t* src, const int64_t* offsets, const int32_t* hwc, int B, int S,
                                 const float* params, int train, const float* mean3, const float* std3, float* out,
                                 fer_stream_t stream) {
  if (B <= 0) return 0;
  if (S <= 0 || S > IMG_MAXS || !mean3 || !std3) return set_error("image_augment: bad size or normalisation");
  if (train && !params) return set_error("image_augment: train mode needs the parameter records");
  hipLaunchKernelGGL(image_augment_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, src, offsets, hwc, S, out,
                     params, train, mean3[0], mean3[1], mean3[2], std3[0], std3[1], std3[2]);
  return hip_check("image_augment");
}
