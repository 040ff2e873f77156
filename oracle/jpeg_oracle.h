/*
 * jpeg_oracle.h -- CPU restatement of SPDL's JPEG -> RGB path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or as the timed CPU baseline).  The product path (spdl_amd) never links,
 * loads or calls it.
 *
 * What it restates (citations relative to the SPDL reference tree):
 *   - demux + FFmpeg `mjpeg` decode called from
 *       src/libspdl/core/detail/ffmpeg/decoder.cpp:50-63 (avcodec_send_packet /
 *       avcodec_receive_frame) with threads=1 (ctx_utils.cpp:180-183);
 *     the arithmetic is FFmpeg's (third-party, not vendored in the reference,
 *     CI pin conda-forge ffmpeg==8.0, .github/workflows/_build_linux.yml:127):
 *       marker parse, baseline Huffman decode with DC prediction, dequant
 *       (block[j] = level * qtab[i]), 8-bit `simple_idct` (idctRowCondDC +
 *       idctSparseColPut), clamp to u8, planes in yuvj4xxp.
 *   - the filter graph of load_image_batch (src/spdl/io/_composite.py:438-443,
 *     src/spdl/io/_preprocessing.py:214-234): scale (force_original_aspect_ratio
 *     decrease|increase) + centred pad / crop + format=rgb24.
 *   - the ImageNet normalisation epilogue (examples/imagenet_classification.py:
 *     96-106): x.float()/255, (x-mean)/std.
 *
 * Parity pinning (see DESIGN.md "Oracle"):
 *   - entropy decode + dequant: pinned bit-exact against IJG libjpeg 9d
 *     (jpeg_read_coefficients), tests/golden/ coefficient fixtures.
 *   - JO_IDCT_ISLOW + nearest chroma + JFIF integer colour conversion: pinned
 *     bit-exact end-to-end against libjpeg 9d (dct_method=JDCT_ISLOW,
 *     do_fancy_upsampling=FALSE).
 *   - JO_IDCT_SIMPLE (FFmpeg simple_idct) and the swscale scale / colour
 *     conversion (sws_oracle.c): parity UNPINNED against FFmpeg (no FFmpeg in
 *     this image); restated from the published algorithm.
 */
#ifndef SPDL_JPEG_ORACLE_H
#define SPDL_JPEG_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  JO_OK = 0,
  JO_ERR_NOT_JPEG = 1,
  JO_ERR_UNSUPPORTED = 2,   /* arithmetic / lossless / 12-bit / CMYK ...   */
  JO_ERR_BAD_HEADER = 3,
  JO_ERR_BAD_HUFFMAN = 4,   /* invalid code / run past coefficient 63     */
  JO_ERR_TRUNCATED = 5,     /* entropy data ended before the last MCU      */
  JO_ERR_BAD_RESTART = 6,
  JO_ERR_BAD_GEOMETRY = 7,
};

enum { JO_IDCT_SIMPLE = 0, JO_IDCT_ISLOW = 1 };

/* pixel formats: planar (CHW) vs interleaved (HWC), channel order */
enum { JO_FMT_RGB = 0, JO_FMT_BGR = 1, JO_FMT_RGB24 = 2, JO_FMT_BGR24 = 3 };

enum { JO_ASPECT_NONE = 0, JO_ASPECT_DECREASE = 1, JO_ASPECT_INCREASE = 2 };
enum { JO_FILTER_BICUBIC = 0, JO_FILTER_BILINEAR = 1, JO_FILTER_LANCZOS = 2 };
enum { JO_DTYPE_U8 = 0, JO_DTYPE_F16 = 1, JO_DTYPE_BF16 = 2 };

#define JO_MAX_COMP 4
#define JO_MAX_BPM 10
/* dequantised DC predictor start value (FFmpeg mjpegdec: 4 << bits) */
#define JO_DC_BIAS 1024

typedef struct {
  int width, height;
  int ncomp;                 /* 1, 3 or 4 (Adobe CMYK / YCCK, all components 1x1) */
  int hmax, vmax;
  int mcux, mcuy;            /* MCUs per row / column */
  int bpm;                   /* blocks per MCU */
  int nblocks;               /* mcux * mcuy * bpm */
  int restart_interval;      /* MCUs per restart interval, 0 = none */
  int comp_h[JO_MAX_COMP], comp_v[JO_MAX_COMP], comp_tq[JO_MAX_COMP];
  int comp_td[JO_MAX_COMP], comp_ta[JO_MAX_COMP];
  int comp_bw[JO_MAX_COMP], comp_bh[JO_MAX_COMP];   /* blocks per row / col */
  int comp_w[JO_MAX_COMP], comp_h_px[JO_MAX_COMP];  /* true plane dims     */
  int mcu_comp[JO_MAX_BPM], mcu_dx[JO_MAX_BPM], mcu_dy[JO_MAX_BPM];
  uint16_t qt[4][64];        /* zig-zag order, as in the stream */
  uint8_t dc_bits[4][17], dc_vals[4][256];
  uint8_t ac_bits[4][17], ac_vals[4][256];
  size_t scan_start;         /* byte offset of the entropy-coded data */
  int progressive;           /* SOF2 */
  int multiscan;             /* the image takes more than one scan (progressive,
                                or sequential with non-interleaved scans):
                                jo_decode_coefs walks every scan */
  int adobe;                 /* APP14 "Adobe" transform flag (0 RGB / CMYK,
                                1 YCbCr, 2 YCCK), -1 without the marker */
  int color;                 /* JO_COLOR_*: the frame's colour model (jo_frame_color) */
} jo_info;

enum { JO_COLOR_GRAY = 0, JO_COLOR_YCBCR = 1, JO_COLOR_RGB = 2, JO_COLOR_CMYK = 3,
       JO_COLOR_YCCK = 4, JO_COLOR_YCBCRK = 5 };
int jo_frame_color(const jo_info* info, const int* comp_id, int* color);

typedef struct {
  int fit_w, fit_h;          /* scale box; <=0 means "input size" */
  int aspect;                /* JO_ASPECT_* */
  int pad_w, pad_h;          /* canvas; <=0 means no pad */
  int crop_w, crop_h;        /* centre crop; <=0 means no crop */
  int filter;                /* JO_FILTER_* */
} jo_resize;

typedef struct {
  int sw, sh;                /* scaled content size */
  int dx, dy;                /* out(x,y) = content(x-dx, y-dy) */
  int ow, oh;                /* output size */
} jo_geom;

const char* jo_strerror(int code);

int jo_parse(const uint8_t* data, size_t size, jo_info* info);

/* Quick SOF probe: width/height/ncomp without full validation. */
int jo_get_image_info(const uint8_t* data, size_t size, int* w, int* h, int* ncomp);

/* Entropy decode + dequant.  coefs: nblocks*64 int16, natural order, MCU order,
 * dequantised FFmpeg-style (DC carries the +1024 level-shift bias).  levels (optional): quantised levels laid out per
 * component in block-raster order (comp 0 first), natural order -- the layout
 * libjpeg's jpeg_read_coefficients exposes, used for pinning. */
int jo_decode_coefs(const uint8_t* data, size_t size, const jo_info* info,
                    int16_t* coefs, int16_t* levels);

void jo_idct_simple(const int16_t* in, uint8_t* out, int stride);
void jo_idct_islow(const int16_t* in, uint8_t* out, int stride);

/* Decoded planes, padded to whole blocks: plane c is comp_bw[c]*8 wide and
 * comp_bh[c]*8 tall, stored back to back. */
size_t jo_planes_size(const jo_info* info);
int jo_decode_planes(const uint8_t* data, size_t size, int idct, uint8_t* planes);

/* Full-resolution RGB through the swscale restatement (JO_CSC_SWSCALE). */
int jo_decode_rgb(const uint8_t* data, size_t size, int idct, int fmt, uint8_t* out);

int jo_geometry(int w, int h, const jo_resize* rs, jo_geom* g);

/* Decode + resize + csc + pad/crop (+ normalise when dtype == F16).
 * out is ow*oh*3 elements (u8 or IEEE fp16 bits). */
int jo_decode_resize(const uint8_t* data, size_t size, int idct, const jo_resize* rs,
                     int fmt, int dtype, const float* mean, const float* stdv,
                     void* out, jo_geom* geom_out);

/* Same, starting from already-decoded planes (used by tests to isolate the
 * resize stage). */
int jo_resize_planes(const jo_info* info, const uint8_t* planes, const jo_resize* rs,
                     int fmt, int dtype, const float* mean, const float* stdv,
                     void* out, jo_geom* geom_out);

/* ---- libswscale restatement (sws_oracle.c) ------------------------------ */

/* colour conversion of the RGB outputs: the reference CPU path's swscale
 * (default), or IJG libjpeg's JFIF integer tables with nearest chroma
 * (full resolution only; pinned against libjpeg 9d) */
enum { JO_CSC_SWSCALE = 0, JO_CSC_JFIF = 1 };

typedef struct {
  int size;       /* taps per output sample */
  int n;          /* output samples */
  int32_t* pos;   /* first source sample of each output */
  int16_t* coef;  /* n * size taps, normalised to `one` */
} jo_sws_filter;

typedef struct {
  int srcW, srcH, dstW, dstH;
  int chrSrcW, chrSrcH, chrDstW, chrDstH;
  int chr_src_hsub, chr_src_vsub;
  int full;              /* SWS_FULL_CHR_H_INT in effect */
  int gray;
  int gbr;               /* three RGB planes through the luma filters */
  int unscaled_special;  /* yuv2rgb_c_24_rgb (nearest chroma) */
  jo_sws_filter hl, hc, vl, vc;
  int32_t crv, cbu, cgu, cgv;                  /* table increments (cy-scaled) */
  int32_t y_coeff, y_offset, v2r, v2g, u2g, u2b; /* yuv2rgb_write_full */
} jo_sws;

int jo_sws_init_filter(int xInc, int srcW, int dstW, int filterAlign, int one, int kind, int srcPos,
                  int dstPos, jo_sws_filter* out);
void jo_sws_filter_free(jo_sws_filter* f);
int jo_sws_init(jo_sws* s, int srcW, int srcH, int hsub, int vsub, int gray, int dstW, int dstH,
                int kind);
void jo_sws_free(jo_sws* s);
int jo_sws_scale(const jo_sws* s, const uint8_t* const* planes, const int* stride, uint8_t* rgb);

/* Full-resolution RGB with a chosen colour conversion (JO_CSC_*). */
int jo_decode_rgb_csc(const uint8_t* data, size_t size, int idct, int csc, int fmt, uint8_t* out);

/* Test helper: the filter swscale builds for one axis (kind = JO_FILTER_*,
 * align 4/2, one 1<<14 / 1<<12, positions as get_local_pos returns them).
 * Writes n positions and n*size taps (cap taps max); returns size or -1. */
int jo_sws_axis(int src, int dst, int kind, int align, int one, int src_pos, int dst_pos,
                int32_t* pos, int16_t* coef, int cap);

uint16_t jo_f32_to_f16(float f);
uint16_t jo_f32_to_bf16(float f);

/* Multi-threaded batch (CPU baseline).  Image i goes to out + i*out_stride
 * bytes.  status[i] receives the per-image code.  Returns #failed. */
void jo_nv12_to_rgb(const uint8_t* src, int frames, int height, int width, int bgr, int coeff,
                    uint8_t* dst);
int jo_decode_resize_batch(const uint8_t* const* data, const size_t* sizes, int n,
                           int idct, const jo_resize* rs, int fmt, int dtype,
                           const float* mean, const float* stdv,
                           uint8_t* out, size_t out_stride, int nthreads, int* status);

int jo_decode_rgb_batch(const uint8_t* const* data, const size_t* sizes, int n,
                        int idct, int fmt, uint8_t* out, size_t out_stride,
                        int nthreads, int* status);

#ifdef __cplusplus
}
#endif
#endif
