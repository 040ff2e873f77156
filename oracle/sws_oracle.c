/*
 * sws_oracle.c -- CPU restatement of the libswscale conversion behind the
 * reference's image filter graph (TEST INFRASTRUCTURE ONLY; see
 * jpeg_oracle.h for who may load it).
 *
 * Reference call sites: the filter graph SPDL builds for load_image /
 * load_image_batch (src/spdl/io/_preprocessing.py:214-254, default
 * "scale=w=224:h=224:flags=bicubic:force_original_aspect_ratio=decrease,
 * pad=...,format=pix_fmts=rgb24") runs in FilterGraphImpl::filter
 * (src/libspdl/core/detail/ffmpeg/filter_graph.cpp:152-178,280-313).  The
 * pad/crop/format filters negotiate rgb24 onto the scale filter's output, so
 * ONE swscale context converts the decoder's yuvj4xxp frame to the scaled
 * rgb24 image; pad (black) and crop then only move pixels.  Without a scale
 * filter ("format=pix_fmts=rgb24") libavfilter inserts a scaler of the same
 * size.
 *
 * The arithmetic is third-party FFmpeg (not vendored in the reference; CI
 * pin conda-forge ffmpeg==8.0, .github/workflows/_build_linux.yml:127), restated
 * here from libswscale's published algorithm (x86-64 build: horizontal filter
 * alignment 4, vertical 2; no SWS_ACCURATE_RND / SWS_BITEXACT, dither auto):
 *   - sws_init_context (libswscale/utils.c): lumXInc/chrXInc, forced full
 *     chroma interpolation for odd dstW or unsubsampled chroma, chroma sizes
 *     AV_CEIL_RSHIFT, get_local_pos() chroma siting (default -513 -> centred);
 *   - initFilter (utils.c): fixed-point bicubic (B = 0, C = 0.6, int64),
 *     bilinear and lanczos (p = 3) kernels, the 0.002 reduce cut-off with the
 *     monotonicity guard, alignment, edge folding ("fix borders"), and the
 *     error-diffusing normalisation to `one` (1<<14 horizontal, 1<<12
 *     vertical);
 *   - hScale8To15_c (swscale.c): (sum >> 7) capped at 32767;
 *   - the RGB24 output writers of libswscale/output.c: yuv2rgb_{X,2,1}_c
 *     (half-width chroma, table lookups) and yuv2rgb_full_{X,2,1}_c +
 *     yuv2rgb_write_full (full chroma), selected per output row as
 *     packed_vscale (vscale.c) does from the vertical filter sizes;
 *   - ff_yuv2rgb_c_init_tables (yuv2rgb.c): BT.601 coefficients
 *     ff_yuv2rgb_coeffs[SWS_CS_ITU601] = {104597, 132201, 25675, 53279},
 *     full-range rescale by 224/255, roundToInt16 13-bit coefficients,
 *     then the cy-rescaled table increments;
 *   - the unscaled yuv420p/yuv422p -> rgb24 converter (yuv2rgb_c_24_rgb,
 *     ff_get_unscaled_swscale): nearest chroma, same tables.
 * Parity is UNPINNED against FFmpeg itself (no FFmpeg in this image or on
 * the GPU box); see DESIGN.md section 4 for the stated assumptions.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "jpeg_oracle.h"

#define SWS_MAX_REDUCE_CUTOFF 0.002
#define SWS_MAX_FILTER_SIZE 256

static int64_t rounded_div(int64_t a, int64_t b) {
  return (a >= 0 ? a + (b >> 1) : a - (b >> 1)) / b;
}

static int log2_floor(unsigned v) {  /* av_log2, av_log2(0) == 0 */
  int n = 0;
  while (v > 1) {
    v >>= 1;
    n++;
  }
  return n;
}

static int64_t abs64(int64_t v) { return v < 0 ? -v : v; }

/* libswscale/utils.c initFilter.  Returns 0, or -1 when swscale would need a
 * cascaded context (filter too long) or an allocation fails. */
int jo_sws_init_filter(int xInc, int srcW, int dstW, int filterAlign, int one, int kind, int srcPos,
                  int dstPos, jo_sws_filter* out) {
  memset(out, 0, sizeof(*out));
  const int64_t fone = 1LL << (54 - (log2_floor((unsigned)(srcW / dstW)) < 8
                                          ? log2_floor((unsigned)(srcW / dstW)) : 8));
  int32_t* pos = (int32_t*)malloc(sizeof(int32_t) * (dstW + 3));
  int64_t* filter = NULL;
  int filterSize;
  if (!pos) return -1;
  if (abs64((int64_t)xInc - 0x10000) < 10 && srcPos == dstPos) {  /* unscaled */
    filterSize = 1;
    filter = (int64_t*)calloc((size_t)dstW, sizeof(int64_t));
    if (!filter) goto fail;
    for (int i = 0; i < dstW; i++) {
      filter[i] = fone;
      pos[i] = i;
    }
  } else {
    int sizeFactor = kind == JO_FILTER_BILINEAR ? 2 : kind == JO_FILTER_LANCZOS ? 6 : 4;
    if (xInc <= 1 << 16)
      filterSize = 1 + sizeFactor;  /* upscale */
    else
      filterSize = 1 + (sizeFactor * srcW + dstW - 1) / dstW;
    if (filterSize > srcW - 2) filterSize = srcW - 2;
    if (filterSize < 1) filterSize = 1;
    filter = (int64_t*)malloc(sizeof(int64_t) * (size_t)dstW * filterSize);
    if (!filter) goto fail;
    int64_t xDstInSrc = ((dstPos * (int64_t)xInc) >> 7) - ((srcPos * 0x10000LL) >> 7);
    for (int i = 0; i < dstW; i++) {
      int xx = (int)((xDstInSrc - (filterSize - 2) * (1LL << 16)) / (1 << 17));
      pos[i] = xx;
      for (int j = 0; j < filterSize; j++) {
        int64_t d = abs64(((int64_t)xx * (1 << 17)) - xDstInSrc) << 13;
        int64_t coeff;
        if (xInc > 1 << 16) d = d * dstW / srcW;
        double floatd = d * (1.0 / (1 << 30));
        if (kind == JO_FILTER_BICUBIC) {
          const int64_t B = (int64_t)(0.0 * (1 << 24));
          const int64_t C = (int64_t)(0.6 * (1 << 24));
          if (d >= 1LL << 31) {
            coeff = 0;
          } else {
            int64_t dd = (d * d) >> 30;
            int64_t ddd = (dd * d) >> 30;
            if (d < 1LL << 30)
              coeff = (12 * (1 << 24) - 9 * B - 6 * C) * ddd +
                      (-18 * (1 << 24) + 12 * B + 6 * C) * dd + (6 * (1 << 24) - 2 * B) * (1 << 30);
            else
              coeff = (-B - 6 * C) * ddd + (6 * B + 30 * C) * dd + (-12 * B - 48 * C) * d +
                      (8 * B + 24 * C) * (1 << 30);
          }
          coeff /= (1LL << 54) / fone;
        } else if (kind == JO_FILTER_LANCZOS) {
          const double p = 3.0;
          coeff = (int64_t)((d ? sin(floatd * M_PI) * sin(floatd * M_PI / p) /
                                     (floatd * floatd * M_PI * M_PI / p)
                               : 1.0) *
                            fone);
          if (floatd > p) coeff = 0;
        } else {  /* bilinear */
          coeff = (1 << 30) - d;
          if (coeff < 0) coeff = 0;
          coeff *= fone >> 30;
        }
        filter[(size_t)i * filterSize + j] = coeff;
        xx++;
      }
      xDstInSrc += 2LL * xInc;
    }
  }
  {
    /* no source / destination filter vectors: filter2 == filter */
    const int f2 = filterSize;
    int minFilterSize = 0;
    for (int i = dstW - 1; i >= 0; i--) {
      int min = f2;
      int64_t cutOff = 0;
      int64_t* row = filter + (size_t)i * f2;
      for (int j = 0; j < f2; j++) {
        cutOff += abs64(row[0]);
        if (cutOff > SWS_MAX_REDUCE_CUTOFF * fone) break;
        if (i < dstW - 1 && pos[i] >= pos[i + 1]) break;  /* keep positions monotonic */
        int k;
        for (k = 1; k < f2; k++) row[k - 1] = row[k];
        row[k - 1] = 0;
        pos[i]++;
      }
      cutOff = 0;
      for (int j = f2 - 1; j > 0; j--) {
        cutOff += abs64(row[j]);
        if (cutOff > SWS_MAX_REDUCE_CUTOFF * fone) break;
        min--;
      }
      if (min > minFilterSize) minFilterSize = min;
    }
    /* x86 (MMX) build: an unscaled vertical filter is not padded to 2 */
    if (minFilterSize == 1 && filterAlign == 2) filterAlign = 1;
    const int fs = (minFilterSize + (filterAlign - 1)) & ~(filterAlign - 1);
    if (fs >= SWS_MAX_FILTER_SIZE) goto fail;  /* swscale: RETCODE_USE_CASCADE */
    int64_t* flt = (int64_t*)calloc((size_t)dstW * fs, sizeof(int64_t));
    if (!flt) goto fail;
    for (int i = 0; i < dstW; i++)
      for (int j = 0; j < fs; j++) flt[(size_t)i * fs + j] = j >= f2 ? 0 : filter[(size_t)i * f2 + j];
    free(filter);
    filter = flt;
    /* fix borders: fold taps outside [0, srcW) into the edge samples */
    for (int i = 0; i < dstW; i++) {
      int64_t* row = filter + (size_t)i * fs;
      if (pos[i] < 0) {
        for (int j = 1; j < fs; j++) {
          int left = j + pos[i] > 0 ? j + pos[i] : 0;
          row[left] += row[j];
          row[j] = 0;
        }
        pos[i] = 0;
      }
      if (pos[i] + fs > srcW) {
        int shift = pos[i] + (fs - srcW < 0 ? fs - srcW : 0);
        int64_t acc = 0;
        for (int j = fs - 1; j >= 0; j--) {
          if (pos[i] + j >= srcW) {
            acc += row[j];
            row[j] = 0;
          }
        }
        for (int j = fs - 1; j >= 0; j--) row[j] = j < shift ? 0 : row[j - shift];
        pos[i] -= shift;
        row[srcW - 1 - pos[i]] += acc;
      }
    }
    out->coef = (int16_t*)malloc(sizeof(int16_t) * (size_t)dstW * fs);
    if (!out->coef) goto fail;
    /* normalise to `one`, carrying the rounding error to the next tap */
    for (int i = 0; i < dstW; i++) {
      const int64_t* row = filter + (size_t)i * fs;
      int64_t error = 0, sum = 0;
      for (int j = 0; j < fs; j++) sum += row[j];
      sum = (sum + one / 2) / one;
      if (!sum) sum = 1;
      for (int j = 0; j < fs; j++) {
        int64_t v = row[j] + error;
        int intV = (int)rounded_div(v, sum);
        out->coef[(size_t)i * fs + j] = (int16_t)intV;
        error = v - (int64_t)intV * sum;
      }
    }
    out->size = fs;
    out->n = dstW;
    out->pos = pos;
    free(filter);
    return 0;
  }
fail:
  free(pos);
  free(filter);
  memset(out, 0, sizeof(*out));
  return -1;
}

void jo_sws_filter_free(jo_sws_filter* f) {
  free(f->pos);
  free(f->coef);
  memset(f, 0, sizeof(*f));
}

/* utils.c get_local_pos: chroma sample position in 1/256 of a destination
 * sample (-513 = unset -> centred between the luma samples it covers). */
static int local_pos(int chr_subsample, int pos) {
  if (pos == -1 || pos <= -513) pos = (128 << chr_subsample) - 128;
  pos += 128;
  return pos >> chr_subsample;
}

static int ceil_rshift(int a, int b) { return -((-a) >> b); }

/* ---- yuv2rgb tables (yuv2rgb.c ff_yuv2rgb_c_init_tables, 24 bpp) -------- */
static int16_t round_to_int16(int64_t f) {  /* utils.c roundToInt16 */
  int r = (int)((f + (1 << 15)) >> 16);
  if (r < -0x7FFF) return (int16_t)0x8000;
  if (r > 0x7FFF) return 0x7FFF;
  return (int16_t)r;
}

static void init_csc(jo_sws* s) {
  /* ff_yuv2rgb_coeffs[SWS_CS_ITU601] (BT.470BG / SMPTE170M / unspecified) */
  int64_t crv = 104597, cbu = 132201, cgu = -25675, cgv = -53279;
  int64_t cy = 1 << 16, oy = 0;
  const int64_t contrast = 1 << 16, saturation = 1 << 16, brightness = 0;
  /* full range (yuvj*: srcRange = 1) */
  crv = (crv * 224) / 255;
  cbu = (cbu * 224) / 255;
  cgu = (cgu * 224) / 255;
  cgv = (cgv * 224) / 255;
  cy = (cy * contrast) >> 16;
  crv = (crv * contrast * saturation) >> 32;
  cbu = (cbu * contrast * saturation) >> 32;
  cgu = (cgu * contrast * saturation) >> 32;
  cgv = (cgv * contrast * saturation) >> 32;
  oy -= 256LL * brightness;
  s->y_coeff = round_to_int16(cy * (1 << 13));
  s->y_offset = round_to_int16(oy * (1 << 9));
  s->v2r = round_to_int16(crv * (1 << 13));
  s->v2g = round_to_int16(cgv * (1 << 13));
  s->u2g = round_to_int16(cgu * (1 << 13));
  s->u2b = round_to_int16(cbu * (1 << 13));
  /* scale coefficients by cy (table increments) */
  s->crv = (int32_t)(((crv * (1 << 16)) + 0x8000) / (cy > 1 ? cy : 1));
  s->cbu = (int32_t)(((cbu * (1 << 16)) + 0x8000) / (cy > 1 ? cy : 1));
  s->cgu = (int32_t)(((cgu * (1 << 16)) + 0x8000) / (cy > 1 ? cy : 1));
  s->cgv = (int32_t)(((cgv * (1 << 16)) + 0x8000) / (cy > 1 ? cy : 1));
  /* y_table[i] = clip((yb + 0x8000) >> 16) with yb stepping by cy from
   * -(384 << 16) - HEADROOM*cy - oy: with cy == 1 << 16 and oy == 0 a lookup
   * at Y + delta reads clip(Y + delta) (asserted below) */
}

static inline int clip8(int v) { return v < 0 ? 0 : v > 255 ? 255 : v; }

/* fill_table / fill_gv_table entry: the offset a chroma value adds to the
 * luma index of the clipping table */
static inline int tab_off(int64_t inc, int c) {
  return (int)(((int64_t)clip8(c) * inc) >> 16) - (int)(inc >> 9);
}

/* yuv2rgb_write (RGB24) through the tables: Y may lie outside [0, 255] */
static inline void table_rgb(const jo_sws* s, int Y, int U, int V, uint8_t* rgb) {
  rgb[0] = (uint8_t)clip8(Y + tab_off(s->crv, V));
  rgb[1] = (uint8_t)clip8(Y + tab_off(s->cgu, U) + tab_off(s->cgv, V));
  rgb[2] = (uint8_t)clip8(Y + tab_off(s->cbu, U));
}

static inline int clip_uintp2_30(int a) {
  if (a & ~((1 << 30) - 1)) return (~a) >> 31 & ((1 << 30) - 1);
  return a;
}

/* output.c yuv2rgb_write_full, RGB24 */
static inline void full_rgb(const jo_sws* s, int Y, int U, int V, uint8_t* rgb) {
  Y -= s->y_offset;
  Y *= s->y_coeff;
  Y += 1 << 21;
  int R = (int)((unsigned)Y + (unsigned)V * (unsigned)s->v2r);
  int G = (int)((unsigned)Y + (unsigned)V * (unsigned)s->v2g + (unsigned)U * (unsigned)s->u2g);
  int B = (int)((unsigned)Y + (unsigned)U * (unsigned)s->u2b);
  if ((R | G | B) & 0xC0000000) {
    R = clip_uintp2_30(R);
    G = clip_uintp2_30(G);
    B = clip_uintp2_30(B);
  }
  rgb[0] = (uint8_t)(R >> 22);
  rgb[1] = (uint8_t)(G >> 22);
  rgb[2] = (uint8_t)(B >> 22);
}

/* ---- context ---------------------------------------------------------------- */

int jo_sws_init(jo_sws* s, int srcW, int srcH, int hsub, int vsub, int gray, int dstW, int dstH,
                int kind) {
  memset(s, 0, sizeof(*s));
  s->srcW = srcW;
  s->srcH = srcH;
  s->dstW = dstW;
  s->dstH = dstH;
  s->gray = gray;
  s->chr_src_hsub = gray ? 0 : hsub;
  s->chr_src_vsub = gray ? 0 : vsub;
  init_csc(s);
  const int64_t lumXInc = (((int64_t)srcW << 16) + (dstW >> 1)) / dstW;
  const int64_t lumYInc = (((int64_t)srcH << 16) + (dstH >> 1)) / dstH;
  /* unscaled yuv420p (even height) / yuv422p -> rgb24: the special
   * converter (ff_get_unscaled_swscale -> yuv2rgb_c_24_rgb), nearest
   * chroma.  Odd widths are left to the scaler path here. */
  const int same = srcW == dstW && srcH == dstH;
  if (same && !gray && hsub == 1 && (vsub == 0 || (vsub == 1 && !(dstH & 1))) && !(dstW & 1)) {
    s->unscaled_special = 1;
    s->full = 0;
    s->chrSrcW = ceil_rshift(srcW, hsub);
    s->chrSrcH = ceil_rshift(srcH, vsub);
    s->chrDstW = s->chrSrcW;
    s->chrDstH = dstH;
    jo_sws_filter* f[4] = {&s->hl, &s->hc, &s->vl, &s->vc};
    const int n[4] = {dstW, s->chrDstW, dstH, dstH};
    for (int k = 0; k < 4; k++) {
      f[k]->size = 1;
      f[k]->n = n[k];
      f[k]->pos = (int32_t*)malloc(sizeof(int32_t) * (n[k] + 3));
      f[k]->coef = (int16_t*)malloc(sizeof(int16_t) * (n[k] + 3));
      if (!f[k]->pos || !f[k]->coef) return -1;
      for (int i = 0; i < n[k]; i++) {
        f[k]->pos[i] = k == 3 ? (i >> vsub) : i;
        f[k]->coef[i] = (int16_t)(k < 2 ? 1 << 14 : 1 << 12);
      }
    }
    return 0;
  }
  /* sws_init_context: forced full chroma interpolation */
  s->full = (dstW & 1) || (s->chr_src_hsub == 0 && s->chr_src_vsub == 0);
  const int chrDstHSub = s->full ? 0 : 1;
  s->chrSrcW = ceil_rshift(srcW, s->chr_src_hsub);
  s->chrSrcH = ceil_rshift(srcH, s->chr_src_vsub);
  s->chrDstW = ceil_rshift(dstW, chrDstHSub);
  s->chrDstH = dstH;
  const int64_t chrXInc = (((int64_t)s->chrSrcW << 16) + (s->chrDstW >> 1)) / s->chrDstW;
  const int64_t chrYInc = (((int64_t)s->chrSrcH << 16) + (s->chrDstH >> 1)) / s->chrDstH;
  if (jo_sws_init_filter((int)lumXInc, srcW, dstW, 4, 1 << 14, kind, local_pos(0, 0),
                    local_pos(0, 0), &s->hl) ||
      jo_sws_init_filter((int)lumYInc, srcH, dstH, 2, 1 << 12, kind, local_pos(0, 0),
                    local_pos(0, 0), &s->vl))
    return -1;
  if (!gray) {
    if (jo_sws_init_filter((int)chrXInc, s->chrSrcW, s->chrDstW, 4, 1 << 14, kind,
                      local_pos(s->chr_src_hsub, -513), local_pos(chrDstHSub, -513), &s->hc) ||
        jo_sws_init_filter((int)chrYInc, s->chrSrcH, s->chrDstH, 2, 1 << 12, kind,
                      local_pos(s->chr_src_vsub, -513), local_pos(0, -513), &s->vc))
      return -1;
  }
  return 0;
}

void jo_sws_free(jo_sws* s) {
  jo_sws_filter_free(&s->hl);
  jo_sws_filter_free(&s->hc);
  jo_sws_filter_free(&s->vl);
  jo_sws_filter_free(&s->vc);
}

/* hScale8To15_c */
static void hscale_row(const uint8_t* src, const jo_sws_filter* f, int16_t* dst) {
  for (int i = 0; i < f->n; i++) {
    int val = 0;
    const int16_t* c = f->coef + (size_t)i * f->size;
    for (int j = 0; j < f->size; j++) val += (int)src[f->pos[i] + j] * c[j];
    val >>= 7;
    dst[i] = (int16_t)(val < (1 << 15) - 1 ? val : (1 << 15) - 1);
  }
}

/* The scaled rgb24 image (dstW x dstH x 3) from the decoded planes.
 * planes[c] / stride[c]: component planes (chroma planes absent for gray). */
/* Three RGB planes (a CMYK frame after FFmpeg's in-decoder conversion,
 * GBRAP) each through the luma filters -- hScale8To15, then the vertical
 * taps with the rounding of swscale's 8-bit planar writers (yuv2planeX:
 * (sum + 2^18) >> 19; two-tap: blend >> 19; one tap: (x + 64) >> 7), clipped.
 * swscale itself routes RGB input through its YUV intermediate when it
 * scales: this per-plane filter is the stated substitute (parity UNPINNED). */
static int sws_scale_gbr(const jo_sws* s, const uint8_t* const* planes, const int* stride,
                         uint8_t* rgb) {
  const int W = s->dstW, H = s->dstH;
  int16_t* h[3];
  for (int c = 0; c < 3; c++) {
    h[c] = (int16_t*)malloc(sizeof(int16_t) * (size_t)s->srcH * W);
    if (!h[c]) {
      for (int k = 0; k < c; k++) free(h[k]);
      return -1;
    }
    for (int r = 0; r < s->srcH; r++) hscale_row(planes[c] + (size_t)r * stride[c], &s->hl, h[c] + (size_t)r * W);
  }
  const int lfs = s->vl.size;
  for (int y = 0; y < H; y++) {
    const int16_t* lf = s->vl.coef + (size_t)y * lfs;
    const int lp = s->vl.pos[y];
    const int mode = lfs == 1 ? 1 : lfs == 2 && lf[0] + lf[1] == 4096 && (unsigned)lf[1] <= 4096u ? 2 : 0;
    for (int x = 0; x < W; x++)
      for (int c = 0; c < 3; c++) {
        const int16_t* col = h[c] + x;
        int v;
        if (mode == 0) {
          v = 1 << 18;
          for (int j = 0; j < lfs; j++) v += col[(size_t)(lp + j) * W] * lf[j];
          v >>= 19;
        } else if (mode == 2) {
          v = (col[(size_t)lp * W] * (4096 - lf[1]) + col[(size_t)(lp + 1) * W] * lf[1]) >> 19;
        } else {
          v = (col[(size_t)lp * W] + 64) >> 7;
        }
        rgb[((size_t)y * W + x) * 3 + c] = (uint8_t)clip8(v);
      }
  }
  for (int c = 0; c < 3; c++) free(h[c]);
  return 0;
}

int jo_sws_scale(const jo_sws* s, const uint8_t* const* planes, const int* stride, uint8_t* rgb) {
  if (s->gbr) return sws_scale_gbr(s, planes, stride, rgb);
  const int W = s->dstW, H = s->dstH;
  const int cw = s->gray ? 0 : s->chrDstW;
  int16_t* lum = (int16_t*)malloc(sizeof(int16_t) * (size_t)s->srcH * W);
  int16_t* cu = (int16_t*)malloc(sizeof(int16_t) * ((size_t)s->chrSrcH * cw + 1));
  int16_t* cv = (int16_t*)malloc(sizeof(int16_t) * ((size_t)s->chrSrcH * cw + 1));
  if (!lum || !cu || !cv) {
    free(lum);
    free(cu);
    free(cv);
    return -1;
  }
  /* horizontal pass of every source row (rows beyond the plane are never
   * referenced with a non-zero tap; the border fold keeps taps in range) */
  for (int r = 0; r < s->srcH; r++) hscale_row(planes[0] + (size_t)r * stride[0], &s->hl, lum + (size_t)r * W);
  if (!s->gray)
    for (int r = 0; r < s->chrSrcH; r++) {
      hscale_row(planes[1] + (size_t)r * stride[1], &s->hc, cu + (size_t)r * cw);
      hscale_row(planes[2] + (size_t)r * stride[2], &s->hc, cv + (size_t)r * cw);
    }
  const int lfs = s->vl.size, cfs = s->gray ? 1 : s->vc.size;
  for (int y = 0; y < H; y++) {
    const int16_t* lf = s->vl.coef + (size_t)y * lfs;
    const int16_t* cf = s->gray ? NULL : s->vc.coef + (size_t)y * cfs;
    const int lp = s->vl.pos[y], cp = s->gray ? 0 : s->vc.pos[y];
    /* packed_vscale: which writer this row uses */
    int mode = 0, yalpha = 0, uvalpha = 0;  /* 0 = X, 1 = _1, 2 = _2 */
    if (s->gray) {
      mode = lfs == 1 ? 1 : lfs == 2 && lf[0] + lf[1] == 4096 && (unsigned)lf[1] <= 4096u ? 2 : 0;
      if (mode == 2) yalpha = lf[1];
    } else if (lfs == 1 && cfs == 1) {
      mode = 1;
    } else if (lfs == 1 && cfs == 2 && cf[0] + cf[1] == 4096 && (unsigned)cf[1] <= 4096u) {
      mode = 1;
      uvalpha = cf[1];
    } else if (lfs == 2 && cfs == 2 && lf[0] + lf[1] == 4096 && (unsigned)lf[1] <= 4096u &&
               cf[0] + cf[1] == 4096 && (unsigned)cf[1] <= 4096u) {
      mode = 2;
      yalpha = lf[1];
      uvalpha = cf[1];
    }
    uint8_t* out = rgb + (size_t)y * W * 3;
    for (int x = 0; x < W; x++) {
      const int ci = s->full ? x : x >> 1;
      int Y, U = 0, V = 0;
      if (s->full) {
        /* yuv2rgb_full_{X,2,1}_c_template; gray: chroma rows hold 128 << 7 */
        if (mode == 0) {
          Y = 1 << 9;
          for (int j = 0; j < lfs; j++) Y += lum[(size_t)(lp + j) * W + x] * lf[j];
          Y >>= 10;
          if (!s->gray) {
            U = (1 << 9) - (128 << 19);
            V = (1 << 9) - (128 << 19);
            for (int j = 0; j < cfs; j++) {
              U += cu[(size_t)(cp + j) * cw + ci] * cf[j];
              V += cv[(size_t)(cp + j) * cw + ci] * cf[j];
            }
            U >>= 10;
            V >>= 10;
          }
        } else if (mode == 2) {
          Y = (lum[(size_t)lp * W + x] * (4096 - yalpha) + lum[(size_t)(lp + 1) * W + x] * yalpha) >> 10;
          if (!s->gray) {
            U = (cu[(size_t)cp * cw + ci] * (4096 - uvalpha) + cu[(size_t)(cp + 1) * cw + ci] * uvalpha -
                 (128 << 19)) >> 10;
            V = (cv[(size_t)cp * cw + ci] * (4096 - uvalpha) + cv[(size_t)(cp + 1) * cw + ci] * uvalpha -
                 (128 << 19)) >> 10;
          }
        } else {
          Y = lum[(size_t)lp * W + x] * 4;
          if (!s->gray) {
            const int c1 = uvalpha ? cp + 1 : cp;
            U = (cu[(size_t)cp * cw + ci] * (4096 - uvalpha) + cu[(size_t)c1 * cw + ci] * uvalpha -
                 (128 << 19)) >> 10;
            V = (cv[(size_t)cp * cw + ci] * (4096 - uvalpha) + cv[(size_t)c1 * cw + ci] * uvalpha -
                 (128 << 19)) >> 10;
          }
        }
        full_rgb(s, Y, U, V, out + 3 * x);
      } else {
        /* yuv2rgb_{X,2,1}_c_template: Y per pixel, U/V per pixel pair */
        if (mode == 0) {
          Y = 1 << 18;
          U = 1 << 18;
          V = 1 << 18;
          for (int j = 0; j < lfs; j++) Y += lum[(size_t)(lp + j) * W + x] * lf[j];
          for (int j = 0; j < cfs; j++) {
            U += cu[(size_t)(cp + j) * cw + ci] * cf[j];
            V += cv[(size_t)(cp + j) * cw + ci] * cf[j];
          }
          Y >>= 19;
          U >>= 19;
          V >>= 19;
        } else if (mode == 2) {
          Y = (lum[(size_t)lp * W + x] * (4096 - yalpha) + lum[(size_t)(lp + 1) * W + x] * yalpha) >> 19;
          U = (cu[(size_t)cp * cw + ci] * (4096 - uvalpha) + cu[(size_t)(cp + 1) * cw + ci] * uvalpha) >> 19;
          V = (cv[(size_t)cp * cw + ci] * (4096 - uvalpha) + cv[(size_t)(cp + 1) * cw + ci] * uvalpha) >> 19;
        } else {
          const int c1 = uvalpha ? cp + 1 : cp;
          Y = (lum[(size_t)lp * W + x] + 64) >> 7;
          U = (cu[(size_t)cp * cw + ci] * (4096 - uvalpha) + cu[(size_t)c1 * cw + ci] * uvalpha +
               (128 << 11)) >> 19;
          V = (cv[(size_t)cp * cw + ci] * (4096 - uvalpha) + cv[(size_t)c1 * cw + ci] * uvalpha +
               (128 << 11)) >> 19;
        }
        table_rgb(s, Y, U, V, out + 3 * x);
      }
    }
  }
  free(lum);
  free(cu);
  free(cv);
  return 0;
}
