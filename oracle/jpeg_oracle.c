/*
 * jpeg_oracle.c -- CPU restatement of SPDL's JPEG -> RGB path (test oracle).
 * The scale / colour-conversion stage is restated in sws_oracle.c.
 *
 * TEST INFRASTRUCTURE ONLY (see jpeg_oracle.h).  Compiled with
 * -ffp-contract=off so the float steps (resize weights, normalisation) are the
 * exact IEEE binary32 sequences written here.
 *
 * Reference call sites restated (paths relative to the SPDL tree):
 *   decode:  src/libspdl/core/detail/ffmpeg/decoder.cpp:50-63 -> FFmpeg mjpeg
 *            (libavcodec/mjpegdec.c decode_block / mjpeg_decode_dc, simple_idct
 *            template 8-bit: idctRowCondDC, idctSparseColPut).
 *   convert: src/libspdl/core/detail/ffmpeg/filter_graph.cpp:280-313 ->
 *            libswscale yuvj4xxp -> rgb24 (sws_oracle.c); the IJG JFIF
 *            tables + nearest chroma remain as JO_CSC_JFIF.
 *   resize:  src/spdl/io/_preprocessing.py:214-234 filter string semantics
 *            (scale force_original_aspect_ratio, pad x=-1:y=-1, crop).
 *   norm:    examples/imagenet_classification.py:96-106.
 */
#include "jpeg_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* Per-thread grow-only scratch buffers: the batch driver decodes many images
 * per thread, and fresh multi-MB mallocs per image page-fault under the
 * process-wide mm lock, which serialises the threads. */
static __thread void* tl_buf[12];
static __thread size_t tl_cap[12];
static void* scratch(int slot, size_t n) {
  if (tl_cap[slot] < n) {
    free(tl_buf[slot]);
    tl_buf[slot] = malloc(n);
    tl_cap[slot] = tl_buf[slot] ? n : 0;
  }
  return tl_buf[slot];
}

static const uint8_t kNatural[64 + 16] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

const char* jo_strerror(int code) {
  switch (code) {
    case JO_OK: return "ok";
    case JO_ERR_NOT_JPEG: return "not a JPEG (missing SOI)";
    case JO_ERR_UNSUPPORTED: return "unsupported JPEG (arithmetic/lossless/12-bit/CMYK)";
    case JO_ERR_BAD_HEADER: return "corrupt JPEG header";
    case JO_ERR_BAD_HUFFMAN: return "corrupt entropy-coded data";
    case JO_ERR_TRUNCATED: return "truncated entropy-coded data";
    case JO_ERR_BAD_RESTART: return "restart marker mismatch";
    case JO_ERR_BAD_GEOMETRY: return "invalid resize geometry";
    default: return "unknown error";
  }
}

static int be16(const uint8_t* p) { return (p[0] << 8) | p[1]; }

/* ------------------------------------------------------------------------ */
/* Marker parsing (T.81 B.2; FFmpeg ff_mjpeg_decode_{dqt,dht,sof,sos}).       */
/* ------------------------------------------------------------------------ */

static int check_huff(const uint8_t* bits) {
  /* canonical code space must not overflow (T.81 C.2) */
  int code = 0;
  for (int l = 1; l <= 16; l++) {
    code += bits[l];
    if (code > (1 << l)) return 0;
    code <<= 1;
  }
  return 1;
}

/* The frame's colour model, decided at the SOF as FFmpeg's mjpeg decoder
 * picks the frame's pix_fmt (ff_mjpeg_decode_sof, as recalled; parity
 * UNPINNED for everything but YCbCr / gray): from the Adobe APP14 transform
 * seen so far and the component ids.
 *   1 component                                   gray8        JO_COLOR_GRAY
 *   3, Adobe transform 0 or ids 'R' 'G' 'B'       gbrp         JO_COLOR_RGB
 *      (all components 1x1; FFmpeg upsamples other samplings of it itself:
 *      unsupported here)
 *   3, otherwise                                  yuvj4xxp     JO_COLOR_YCBCR
 *   4 (all components 1x1), Adobe transform 0     gbrap        JO_COLOR_CMYK
 *   4, Adobe transform 2                          yuva444p     JO_COLOR_YCCK
 *   4, other / no marker                          yuva444p     JO_COLOR_YCBCRK
 * (CMYK and YCCK are converted in the decoder: jo_cmyk_transform.) */
int jo_frame_color(const jo_info* info, const int* comp_id, int* color) {
  int all11 = 1;
  for (int c = 0; c < info->ncomp; c++) all11 &= info->comp_h[c] == 1 && info->comp_v[c] == 1;
  if (info->ncomp == 1) {
    *color = JO_COLOR_GRAY;
  } else if (info->ncomp == 3) {
    const int rgb = info->adobe == 0 || (comp_id[0] == 'R' && comp_id[1] == 'G' && comp_id[2] == 'B');
    if (rgb && !all11) return JO_ERR_UNSUPPORTED;
    *color = rgb ? JO_COLOR_RGB : JO_COLOR_YCBCR;
  } else {
    if (!all11) return JO_ERR_UNSUPPORTED;
    *color = info->adobe == 0 ? JO_COLOR_CMYK : info->adobe == 2 ? JO_COLOR_YCCK : JO_COLOR_YCBCRK;
  }
  return JO_OK;
}

int jo_parse(const uint8_t* d, size_t size, jo_info* info) {
  memset(info, 0, sizeof(*info));
  info->adobe = -1;
  if (size < 4 || d[0] != 0xFF || d[1] != 0xD8) return JO_ERR_NOT_JPEG;
  int have_sof = 0, qt_have[4] = {0}, dc_have[4] = {0}, ac_have[4] = {0};
  int comp_id[JO_MAX_COMP] = {0};
  size_t pos = 2;
  for (;;) {
    while (pos < size && d[pos] != 0xFF) pos++; /* skip garbage */
    while (pos < size && d[pos] == 0xFF) pos++; /* fill bytes */
    if (pos >= size) return JO_ERR_BAD_HEADER;
    int m = d[pos++];
    if (m == 0xD8 || m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;
    if (m == 0xD9) return JO_ERR_BAD_HEADER; /* EOI before SOS */
    if (pos + 2 > size) return JO_ERR_BAD_HEADER;
    int len = be16(d + pos);
    if (len < 2 || pos + (size_t)len > size) return JO_ERR_BAD_HEADER;
    const uint8_t* s = d + pos + 2;
    int n = len - 2;
    pos += (size_t)len;
    if (m == 0xDB) { /* DQT */
      while (n > 0) {
        int pq = s[0] >> 4, tq = s[0] & 15;
        if (tq > 3 || pq > 1) return JO_ERR_BAD_HEADER;
        int need = 1 + 64 * (pq + 1);
        if (n < need) return JO_ERR_BAD_HEADER;
        for (int i = 0; i < 64; i++)
          info->qt[tq][i] = pq ? (uint16_t)be16(s + 1 + 2 * i) : s[1 + i];
        qt_have[tq] = 1;
        s += need;
        n -= need;
      }
    } else if (m == 0xC4) { /* DHT */
      while (n > 0) {
        if (n < 17) return JO_ERR_BAD_HEADER;
        int tc = s[0] >> 4, th = s[0] & 15;
        if (tc > 1 || th > 3) return JO_ERR_BAD_HEADER;
        uint8_t bits[17];
        bits[0] = 0;
        int total = 0;
        for (int l = 1; l <= 16; l++) { bits[l] = s[l]; total += s[l]; }
        if (total > 256 || n < 17 + total || !check_huff(bits)) return JO_ERR_BAD_HEADER;
        uint8_t* dbits = tc ? info->ac_bits[th] : info->dc_bits[th];
        uint8_t* dvals = tc ? info->ac_vals[th] : info->dc_vals[th];
        memcpy(dbits, bits, 17);
        memset(dvals, 0, 256);
        memcpy(dvals, s + 17, (size_t)total);
        (tc ? ac_have : dc_have)[th] = 1;
        s += 17 + total;
        n -= 17 + total;
      }
    } else if (m == 0xC0 || m == 0xC1 || m == 0xC2) { /* SOF0/1 sequential, SOF2 progressive */
      info->progressive = m == 0xC2;
      if (n < 6) return JO_ERR_BAD_HEADER;
      if (s[0] != 8) return JO_ERR_UNSUPPORTED;
      info->height = be16(s + 1);
      info->width = be16(s + 3);
      int nf = s[5];
      if (info->height == 0) return JO_ERR_UNSUPPORTED; /* DNL */
      if (info->width == 0) return JO_ERR_BAD_HEADER;
      if (nf != 1 && nf != 3 && nf != 4) return JO_ERR_UNSUPPORTED;
      if (n < 6 + 3 * nf) return JO_ERR_BAD_HEADER;
      info->ncomp = nf;
      for (int c = 0; c < nf; c++) {
        comp_id[c] = s[6 + 3 * c];
        info->comp_h[c] = s[7 + 3 * c] >> 4;
        info->comp_v[c] = s[7 + 3 * c] & 15;
        info->comp_tq[c] = s[8 + 3 * c];
        if (info->comp_h[c] < 1 || info->comp_h[c] > 4 || info->comp_v[c] < 1 ||
            info->comp_v[c] > 4 || info->comp_tq[c] > 3)
          return JO_ERR_BAD_HEADER;
      }
      int rc = jo_frame_color(info, comp_id, &info->color);
      if (rc) return rc;
      have_sof = 1;
    } else if (m == 0xC3 || (m >= 0xC5 && m <= 0xC7) || (m >= 0xC9 && m <= 0xCB) ||
               (m >= 0xCD && m <= 0xCF)) {
      return JO_ERR_UNSUPPORTED; /* lossless, hierarchical, arithmetic */
    } else if (m == 0xEE) { /* APP14: Adobe's transform flag (in effect from the next SOF) */
      if (n >= 12 && memcmp(s, "Adobe", 5) == 0) info->adobe = s[11];
    } else if (m == 0xDD) { /* DRI */
      if (n < 2) return JO_ERR_BAD_HEADER;
      info->restart_interval = be16(s);
    } else if (m == 0xDA) { /* SOS */
      if (!have_sof) return JO_ERR_BAD_HEADER;
      int ns = s[0];
      if (ns < 1 || ns > info->ncomp) return JO_ERR_BAD_HEADER;
      /* progressive, or sequential with non-interleaved scans: the first scan
       * fixes nothing beyond the frame; every scan is walked at decode time */
      info->multiscan = info->progressive || ns != info->ncomp;
      if (n < 1 + 2 * ns + 3) return JO_ERR_BAD_HEADER;
      int order[JO_MAX_COMP];
      for (int i = 0; i < ns; i++) {
        int cs = s[1 + 2 * i], c = -1;
        for (int k = 0; k < info->ncomp; k++)
          if (comp_id[k] == cs) c = k;
        if (c < 0) return JO_ERR_BAD_HEADER;
        order[i] = c;
        info->comp_td[c] = s[2 + 2 * i] >> 4;
        info->comp_ta[c] = s[2 + 2 * i] & 15;
        if (info->comp_td[c] > 3 || info->comp_ta[c] > 3) return JO_ERR_BAD_HEADER;
      }
      int ss = s[1 + 2 * ns], se = s[2 + 2 * ns], ahal = s[3 + 2 * ns];
      if (!info->multiscan && (ss != 0 || se != 63 || ahal != 0)) return JO_ERR_UNSUPPORTED;
      info->scan_start = pos;
      if (info->multiscan) /* blocks of an MCU in frame component order */
        for (int i = 0; i < info->ncomp; i++) order[i] = i;
      /* geometry */
      int hmax = 1, vmax = 1;
      for (int c = 0; c < info->ncomp; c++) {
        if (info->comp_h[c] > hmax) hmax = info->comp_h[c];
        if (info->comp_v[c] > vmax) vmax = info->comp_v[c];
      }
      info->hmax = hmax;
      info->vmax = vmax;
      for (int c = 0; c < info->ncomp; c++) {
        if (hmax % info->comp_h[c] || vmax % info->comp_v[c]) return JO_ERR_UNSUPPORTED;
        if (!info->multiscan && (!qt_have[info->comp_tq[c]] || !dc_have[info->comp_td[c]] ||
                                 !ac_have[info->comp_ta[c]]))
          return JO_ERR_BAD_HEADER;
        info->comp_w[c] = (info->width * info->comp_h[c] + hmax - 1) / hmax;
        info->comp_h_px[c] = (info->height * info->comp_v[c] + vmax - 1) / vmax;
      }
      if (info->ncomp == 1) {
        info->comp_bw[0] = (info->comp_w[0] + 7) / 8;
        info->comp_bh[0] = (info->comp_h_px[0] + 7) / 8;
        info->mcux = info->comp_bw[0];
        info->mcuy = info->comp_bh[0];
        info->bpm = 1;
        info->mcu_comp[0] = 0;
      } else {
        info->mcux = (info->width + 8 * hmax - 1) / (8 * hmax);
        info->mcuy = (info->height + 8 * vmax - 1) / (8 * vmax);
        int b = 0;
        for (int i = 0; i < (info->multiscan ? info->ncomp : ns); i++) {
          int c = order[i];
          info->comp_bw[c] = info->mcux * info->comp_h[c];
          info->comp_bh[c] = info->mcuy * info->comp_v[c];
          for (int y = 0; y < info->comp_v[c]; y++)
            for (int x = 0; x < info->comp_h[c]; x++) {
              if (b >= JO_MAX_BPM) return JO_ERR_UNSUPPORTED;
              info->mcu_comp[b] = c;
              info->mcu_dx[b] = x;
              info->mcu_dy[b] = y;
              b++;
            }
        }
        info->bpm = b;
      }
      info->nblocks = info->mcux * info->mcuy * info->bpm;
      return JO_OK;
    }
    /* APPn, COM, DHP, EXP, DNL, JPG... : skipped */
  }
}

int jo_get_image_info(const uint8_t* d, size_t size, int* w, int* h, int* ncomp) {
  jo_info info;
  int rc = jo_parse(d, size, &info);
  if (rc) return rc;
  *w = info.width;
  *h = info.height;
  *ncomp = info.ncomp;
  return JO_OK;
}

/* ------------------------------------------------------------------------ */
/* Huffman decoding                                                          */
/* ------------------------------------------------------------------------ */

#define LOOKBITS 9
typedef struct {
  int32_t maxcode[18];   /* largest code of length l, -1 if none */
  int32_t valoff[17];    /* index into vals for first code of length l minus that code */
  uint8_t vals[256];
  uint16_t look[1 << LOOKBITS]; /* (len << 8) | sym, 0 when len > LOOKBITS */
} huff_t;

static void build_huff(const uint8_t* bits, const uint8_t* vals, huff_t* h) {
  int code = 0, k = 0;
  memcpy(h->vals, vals, 256);
  memset(h->look, 0, sizeof(h->look));
  for (int l = 1; l <= 16; l++) {
    if (bits[l]) {
      h->valoff[l] = k - code;
      for (int i = 0; i < bits[l]; i++) {
        if (l <= LOOKBITS) {
          int lo = code << (LOOKBITS - l), cnt = 1 << (LOOKBITS - l);
          for (int j = 0; j < cnt; j++) h->look[lo + j] = (uint16_t)((l << 8) | vals[k]);
        }
        code++;
        k++;
      }
      h->maxcode[l] = code - 1;
    } else {
      h->maxcode[l] = -1;
      h->valoff[l] = 0;
    }
    code <<= 1;
  }
  h->maxcode[17] = 0x7FFFFFFF;
}

typedef struct {
  const uint8_t* d;
  size_t size, pos;
  uint64_t buf;
  int cnt;
  int hit_marker;
  int64_t real_bits;   /* bits loaded from actual data */
  int64_t used_bits;   /* bits consumed */
} bitrd_t;

static void br_fill(bitrd_t* b) {
  while (b->cnt <= 56) {
    unsigned byte = 0;
    if (!b->hit_marker) {
      if (b->pos >= b->size) {
        b->hit_marker = 1;
      } else {
        unsigned c = b->d[b->pos];
        if (c == 0xFF) {
          unsigned nx = b->pos + 1 < b->size ? b->d[b->pos + 1] : 0xD9;
          if (nx == 0x00) {
            b->pos += 2;
            byte = 0xFF;
            b->real_bits += 8;
          } else {
            b->hit_marker = 1;
          }
        } else {
          b->pos++;
          byte = c;
          b->real_bits += 8;
        }
      }
    }
    b->buf |= (uint64_t)byte << (56 - b->cnt);
    b->cnt += 8;
  }
}

static inline unsigned br_peek16(bitrd_t* b) {
  if (b->cnt < 32) br_fill(b);
  return (unsigned)(b->buf >> 48);
}
static inline void br_skip(bitrd_t* b, int n) {
  b->buf <<= n;
  b->cnt -= n;
  b->used_bits += n;
}
static inline unsigned br_get(bitrd_t* b, int n) {
  if (n == 0) return 0;
  if (b->cnt < 32) br_fill(b);
  unsigned v = (unsigned)(b->buf >> (64 - n));
  br_skip(b, n);
  return v;
}

/* returns symbol or -1 for an invalid code */
static int huff_decode(bitrd_t* b, const huff_t* h) {
  unsigned w = br_peek16(b);
  unsigned e = h->look[w >> (16 - LOOKBITS)];
  if (e) {
    br_skip(b, (int)(e >> 8));
    return (int)(e & 0xFF);
  }
  for (int l = LOOKBITS + 1; l <= 16; l++) {
    int code = (int)(w >> (16 - l));
    if (code <= h->maxcode[l]) {
      br_skip(b, l);
      return h->vals[h->valoff[l] + code];
    }
  }
  return -1;
}

static inline int extend(unsigned v, int s) {
  return (v < (1u << (s - 1))) ? (int)v - ((1 << s) - 1) : (int)v;
}

static inline int16_t clip16(int32_t v) {
  return v < -32768 ? -32768 : v > 32767 ? 32767 : (int16_t)v;
}

/* ------------------------------------------------------------------------ */
/* Multi-scan images: progressive (SOF2) and sequential with non-interleaved */
/* scans.  Every scan adds to one level accumulator per coefficient (zig-zag */
/* index, per block in MCU order); the levels are dequantised FFmpeg-style at */
/* the end (block[j] = level * q, DC biased by 1024, int16).                 */
/* Scan semantics: T.81 G.1.2 as libjpeg 9d implements them (jdphuff.c      */
/* decode_mcu_DC_first / DC_refine / AC_first / AC_refine; jdhuff.c for the  */
/* sequential scans), which is what tests/golden pins; FFmpeg's mjpegdec     */
/* (decode_dc_progressive, decode_block_progressive, decode_block_refinement)*/
/* computes the same values on valid streams.                                */
/* ------------------------------------------------------------------------ */

typedef struct {
  int ns, comp[JO_MAX_COMP], td[JO_MAX_COMP], ta[JO_MAX_COMP];
  int ss, se, ah, al;
} scan_t;

/* MCU-order block index of component c's block (bx, by) in its block grid */
static size_t ms_block(const jo_info* info, int c, int bx, int by) {
  if (info->ncomp == 1) return (size_t)by * info->mcux + bx;
  int b0 = 0;
  for (int k = 0; k < c; k++) b0 += info->comp_h[k] * info->comp_v[k];
  int mx = bx / info->comp_h[c], my = by / info->comp_v[c];
  int b = b0 + (by % info->comp_v[c]) * info->comp_h[c] + (bx % info->comp_h[c]);
  return ((size_t)my * info->mcux + mx) * info->bpm + b;
}

/* one block of one scan; lev: the block's 64 levels (zig-zag index) */
static int ms_block_decode(bitrd_t* br, const jo_info* info, const scan_t* sc, int progressive,
                           const huff_t* dh, const huff_t* ah, int32_t* pred, int32_t* lev,
                           int* eobrun) {
  if (!progressive) { /* sequential scan: DC + AC of the block */
    int s = huff_decode(br, dh);
    if (s < 0 || s > 15) return JO_ERR_BAD_HUFFMAN;
    *pred += s ? extend(br_get(br, s), s) : 0;
    lev[0] = *pred;
    for (int k = 1; k < 64;) {
      int rs = huff_decode(br, ah);
      if (rs < 0) return JO_ERR_BAD_HUFFMAN;
      int r = rs >> 4;
      s = rs & 15;
      if (s == 0) {
        if (r == 15) { k += 16; continue; }
        if (r != 0) return JO_ERR_BAD_HUFFMAN;
        break;
      }
      k += r;
      if (k > 63) return JO_ERR_BAD_HUFFMAN;
      lev[k++] = extend(br_get(br, s), s);
    }
    return JO_OK;
  }
  const int al = sc->al;
  if (sc->ss == 0) {
    if (sc->ah == 0) { /* DC first: the difference, scaled by 2^Al */
      int s = huff_decode(br, dh);
      if (s < 0 || s > 15) return JO_ERR_BAD_HUFFMAN;
      *pred += s ? extend(br_get(br, s), s) : 0;
      lev[0] = (int32_t)((uint32_t)*pred << al);
    } else if (br_get(br, 1)) { /* DC refine: one bit */
      lev[0] |= 1 << al;
    }
    return JO_OK;
  }
  if (sc->ah == 0) { /* AC first */
    if (*eobrun > 0) {
      (*eobrun)--;
      return JO_OK;
    }
    for (int k = sc->ss; k <= sc->se; k++) {
      int rs = huff_decode(br, ah);
      if (rs < 0) return JO_ERR_BAD_HUFFMAN;
      int r = rs >> 4, s = rs & 15;
      if (s) {
        k += r;
        if (k > sc->se) return JO_ERR_BAD_HUFFMAN;
        lev[k] = (int32_t)((uint32_t)extend(br_get(br, s), s) << al);
      } else if (r == 15) {
        k += 15;
      } else {
        *eobrun = (1 << r) - 1;
        if (r) *eobrun += (int)br_get(br, r);
        break;
      }
    }
    return JO_OK;
  }
  /* AC refine: new coefficients are +-1 at bit Al; every coefficient already
   * non-zero that the scan passes gets one correction bit */
  const int32_t p1 = 1 << al, m1 = -(1 << al);
  int k = sc->ss;
  if (*eobrun <= 0) {
    for (; k <= sc->se; k++) {
      int rs = huff_decode(br, ah);
      if (rs < 0) return JO_ERR_BAD_HUFFMAN;
      int r = rs >> 4, s = rs & 15;
      int32_t v = 0;
      if (s) {
        if (s != 1) return JO_ERR_BAD_HUFFMAN;
        v = br_get(br, 1) ? p1 : m1;
      } else if (r != 15) {
        *eobrun = 1 << r;
        if (r) *eobrun += (int)br_get(br, r);
        break; /* the rest of the block refines below */
      }
      /* skip r zero-history coefficients, refining the non-zero ones */
      for (; k <= sc->se; k++) {
        int32_t* c = &lev[k];
        if (*c != 0) {
          if (br_get(br, 1) && (*c & p1) == 0) *c += *c >= 0 ? p1 : m1;
        } else {
          if (r == 0) break;
          r--;
        }
      }
      if (k > sc->se) {
        if (v) return JO_ERR_BAD_HUFFMAN; /* a new coefficient past Se */
        break;
      }
      if (v) lev[k] = v;
    }
  }
  if (*eobrun > 0) {
    for (; k <= sc->se; k++) {
      int32_t* c = &lev[k];
      if (*c != 0 && br_get(br, 1) && (*c & p1) == 0) *c += *c >= 0 ? p1 : m1;
    }
    (*eobrun)--;
  }
  return JO_OK;
}

/* Decode one scan whose entropy data starts at `pos`; returns the byte
 * position after it (the next marker) in *end. */
static int ms_scan(const uint8_t* d, size_t size, size_t pos, const jo_info* info,
                   const scan_t* sc, int ri, const huff_t* dct, const huff_t* act, int32_t* lev,
                   size_t* end) {
  bitrd_t br;
  memset(&br, 0, sizeof(br));
  br.d = d;
  br.size = size;
  br.pos = pos;
  int32_t pred[JO_MAX_COMP] = {0};
  int eobrun = 0;
  const int prog = info->progressive;
  /* interleaved: MCUs of the frame; one component: its blocks in raster
   * order over its own (unpadded) block grid, one block per MCU */
  int nmcu, bw1 = 0;
  if (sc->ns > 1) {
    nmcu = info->mcux * info->mcuy;
  } else {
    int c = sc->comp[0];
    bw1 = info->ncomp == 1 ? info->mcux : (info->comp_w[c] + 7) / 8;
    int bh1 = info->ncomp == 1 ? info->mcuy : (info->comp_h_px[c] + 7) / 8;
    nmcu = bw1 * bh1;
  }
  for (int mcu = 0; mcu < nmcu; mcu++) {
    if (ri && mcu && mcu % ri == 0) {
      if (br.used_bits > br.real_bits) return JO_ERR_TRUNCATED;
      size_t p = br.pos;
      for (;;) {
        if (p >= size) return JO_ERR_BAD_RESTART;
        if (d[p] == 0xFF && p + 1 < size && d[p + 1] == 0x00) { p += 2; continue; }
        if (d[p] == 0xFF) break;
        p++;
      }
      while (p < size && d[p] == 0xFF) p++;
      if (p >= size || d[p] < 0xD0 || d[p] > 0xD7) return JO_ERR_BAD_RESTART;
      br.pos = p + 1;
      br.buf = 0;
      br.cnt = 0;
      br.hit_marker = 0;
      br.real_bits = br.used_bits = 0;
      for (int c = 0; c < JO_MAX_COMP; c++) pred[c] = 0;
      eobrun = 0;
    }
    for (int i = 0; i < sc->ns; i++) {
      const int c = sc->comp[i];
      const huff_t* dh = &dct[sc->td[i]];
      const huff_t* ah = &act[sc->ta[i]];
      if (sc->ns > 1) {
        int mx = mcu % info->mcux, my = mcu / info->mcux;
        for (int y = 0; y < info->comp_v[c]; y++)
          for (int x = 0; x < info->comp_h[c]; x++) {
            size_t b = ms_block(info, c, mx * info->comp_h[c] + x, my * info->comp_v[c] + y);
            int rc = ms_block_decode(&br, info, sc, prog, dh, ah, &pred[c], lev + b * 64, &eobrun);
            if (rc) return rc;
          }
      } else {
        size_t b = ms_block(info, c, mcu % bw1, mcu / bw1);
        int rc = ms_block_decode(&br, info, sc, prog, dh, ah, &pred[c], lev + b * 64, &eobrun);
        if (rc) return rc;
      }
    }
  }
  if (br.used_bits > br.real_bits) return JO_ERR_TRUNCATED;
  /* the next marker: past the bytes the reader took (stuffed 0xFF00 pairs
   * included), then skip to a marker that is not RSTn */
  size_t p = br.pos;
  for (;;) {
    while (p < size && d[p] != 0xFF) p++;
    if (p + 1 >= size) break;
    if (d[p + 1] == 0x00 || (d[p + 1] >= 0xD0 && d[p + 1] <= 0xD7)) { p += 2; continue; }
    break;
  }
  *end = p;
  return JO_OK;
}

static int ms_decode(const uint8_t* d, size_t size, const jo_info* info, int16_t* coefs,
                     int16_t* levels) {
  int32_t* lev = (int32_t*)calloc((size_t)info->nblocks * 64, sizeof(int32_t));
  if (!lev) return JO_ERR_UNSUPPORTED;
  huff_t dct[4], act[4];
  memset(dct, 0, sizeof(dct));
  memset(act, 0, sizeof(act));
  int comp_id[JO_MAX_COMP] = {0};
  int ri = 0, rc = JO_OK, nscan = 0;
  size_t pos = 2;
  for (;;) {
    while (pos < size && d[pos] != 0xFF) pos++;
    while (pos < size && d[pos] == 0xFF) pos++;
    if (pos >= size) break; /* no EOI: what was decoded stands */
    int m = d[pos++];
    if (m == 0xD8 || m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;
    if (m == 0xD9) break;
    if (pos + 2 > size) { rc = JO_ERR_BAD_HEADER; break; }
    int len = be16(d + pos);
    if (len < 2 || pos + (size_t)len > size) { rc = JO_ERR_BAD_HEADER; break; }
    const uint8_t* s = d + pos + 2;
    int n = len - 2;
    pos += (size_t)len;
    if (m == 0xC4) {
      while (n >= 17) {
        int tc = s[0] >> 4, th = s[0] & 15, total = 0;
        uint8_t bits[17], vals[256];
        bits[0] = 0;
        for (int l = 1; l <= 16; l++) { bits[l] = s[l]; total += s[l]; }
        if (tc > 1 || th > 3 || total > 256 || n < 17 + total || !check_huff(bits)) {
          rc = JO_ERR_BAD_HEADER;
          break;
        }
        memset(vals, 0, sizeof(vals));
        memcpy(vals, s + 17, (size_t)total);
        build_huff(bits, vals, tc ? &act[th] : &dct[th]);
        s += 17 + total;
        n -= 17 + total;
      }
      if (rc) break;
    } else if (m == 0xC0 || m == 0xC1 || m == 0xC2) {
      for (int c = 0; c < info->ncomp && 8 + 3 * c < len; c++) comp_id[c] = s[6 + 3 * c];
    } else if (m == 0xDD) {
      if (n >= 2) ri = be16(s);
    } else if (m == 0xDA) {
      scan_t sc;
      sc.ns = s[0];
      if (sc.ns < 1 || sc.ns > info->ncomp || n < 1 + 2 * sc.ns + 3) { rc = JO_ERR_BAD_HEADER; break; }
      for (int i = 0; i < sc.ns; i++) {
        int cs = s[1 + 2 * i], c = -1;
        for (int k = 0; k < info->ncomp; k++)
          if (comp_id[k] == cs) c = k;
        if (c < 0) { rc = JO_ERR_BAD_HEADER; break; }
        sc.comp[i] = c;
        sc.td[i] = s[2 + 2 * i] >> 4;
        sc.ta[i] = s[2 + 2 * i] & 15;
        if (sc.td[i] > 3 || sc.ta[i] > 3) { rc = JO_ERR_BAD_HEADER; break; }
      }
      if (rc) break;
      sc.ss = s[1 + 2 * sc.ns];
      sc.se = s[2 + 2 * sc.ns];
      sc.ah = s[3 + 2 * sc.ns] >> 4;
      sc.al = s[3 + 2 * sc.ns] & 15;
      if (info->progressive) {
        /* T.81 G.1.1.1.1: DC scans Ss = Se = 0; AC scans one component */
        if (sc.ss > sc.se || sc.se > 63 || sc.al > 13 || (sc.ss == 0 && sc.se != 0) ||
            (sc.ss > 0 && sc.ns != 1)) { rc = JO_ERR_BAD_HEADER; break; }
      } else if (sc.ss != 0 || sc.se != 63 || sc.ah || sc.al) {
        rc = JO_ERR_BAD_HEADER;
        break;
      }
      size_t end = pos;
      rc = ms_scan(d, size, pos, info, &sc, ri, dct, act, lev, &end);
      if (rc) break;
      pos = end;
      nscan++;
    }
  }
  if (!rc && !nscan) rc = JO_ERR_BAD_HEADER;
  if (!rc) {
    for (int b = 0; b < info->nblocks; b++) {
      const int c = info->mcu_comp[b % info->bpm];
      const uint16_t* q = info->qt[info->comp_tq[c]];
      const int32_t* lv = lev + (size_t)b * 64;
      int16_t* blk = coefs + (size_t)b * 64;
      blk[0] = (int16_t)(JO_DC_BIAS + lv[0] * (int32_t)q[0]);
      for (int k = 1; k < 64; k++) blk[kNatural[k]] = (int16_t)(lv[k] * (int32_t)q[k]);
    }
    if (levels) {
      size_t o = 0;
      for (int c = 0; c < info->ncomp; c++) {
        for (int by = 0; by < info->comp_bh[c]; by++)
          for (int bx = 0; bx < info->comp_bw[c]; bx++) {
            const int32_t* lv = lev + ms_block(info, c, bx, by) * 64;
            int16_t* out = levels + o + ((size_t)by * info->comp_bw[c] + bx) * 64;
            for (int k = 0; k < 64; k++) out[kNatural[k]] = (int16_t)lv[k];
          }
        o += (size_t)info->comp_bw[c] * info->comp_bh[c] * 64;
      }
    }
  }
  free(lev);
  return rc;
}

int jo_decode_coefs(const uint8_t* d, size_t size, const jo_info* info, int16_t* coefs,
                    int16_t* levels) {
  if (info->multiscan) {
    memset(coefs, 0, (size_t)info->nblocks * 64 * sizeof(int16_t));
    return ms_decode(d, size, info, coefs, levels);
  }
  huff_t dct[4], act[4];
  for (int t = 0; t < 4; t++) {
    build_huff(info->dc_bits[t], info->dc_vals[t], &dct[t]);
    build_huff(info->ac_bits[t], info->ac_vals[t], &act[t]);
  }
  size_t lvl_off[JO_MAX_COMP] = {0};
  {
    size_t o = 0;
    for (int c = 0; c < info->ncomp; c++) {
      lvl_off[c] = o;
      o += (size_t)info->comp_bw[c] * info->comp_bh[c] * 64;
    }
  }
  memset(coefs, 0, (size_t)info->nblocks * 64 * sizeof(int16_t));
  if (levels) {
    size_t tot = 0;
    for (int c = 0; c < info->ncomp; c++) tot += (size_t)info->comp_bw[c] * info->comp_bh[c] * 64;
    memset(levels, 0, tot * sizeof(int16_t));
  }
  bitrd_t br;
  memset(&br, 0, sizeof(br));
  br.d = d;
  br.size = size;
  br.pos = info->scan_start;
  /* FFmpeg mjpegdec initialises (and resets at each RSTn) the dequantised DC
   * predictor to 4 << bits = 1024: the +128 level shift lives in block[0]. */
  int32_t pred[JO_MAX_COMP] = {0};  /* sum of DC diffs (quantised) */
  uint32_t last_dc[JO_MAX_COMP] = {JO_DC_BIAS, JO_DC_BIAS, JO_DC_BIAS, JO_DC_BIAS};
  int nmcu = info->mcux * info->mcuy;
  int ri = info->restart_interval;
  for (int mcu = 0; mcu < nmcu; mcu++) {
    if (ri && mcu && mcu % ri == 0) {
      /* restart: check the consumed bits were real, drop padding, eat RSTn */
      if (br.used_bits > br.real_bits) return JO_ERR_TRUNCATED;
      /* a segment is the byte run between markers: leftover bits of this
       * interval are ignored, decoding resumes after the next marker, which
       * must be RSTn (same segmentation as the device destuff pass). */
      size_t p = br.pos;
      for (;;) {
        if (p >= size) return JO_ERR_BAD_RESTART;
        if (d[p] == 0xFF && p + 1 < size && d[p + 1] == 0x00) {
          p += 2;
          continue;
        }
        if (d[p] == 0xFF) break;
        p++;
      }
      while (p < size && d[p] == 0xFF) p++;
      if (p >= size || d[p] < 0xD0 || d[p] > 0xD7) return JO_ERR_BAD_RESTART;
      br.pos = p + 1;
      br.buf = 0;
      br.cnt = 0;
      br.hit_marker = 0;
      br.real_bits = br.used_bits = 0;
      for (int c = 0; c < JO_MAX_COMP; c++) pred[c] = 0, last_dc[c] = JO_DC_BIAS;
    }
    int mx = mcu % info->mcux, my = mcu / info->mcux;
    for (int b = 0; b < info->bpm; b++) {
      int c = info->mcu_comp[b];
      const uint16_t* q = info->qt[info->comp_tq[c]];
      int16_t* blk = coefs + ((size_t)mcu * info->bpm + b) * 64;
      int bx, by;
      if (info->ncomp == 1) {
        bx = mx;
        by = my;
      } else {
        bx = mx * info->comp_h[c] + info->mcu_dx[b];
        by = my * info->comp_v[c] + info->mcu_dy[b];
      }
      int16_t* lv = levels ? levels + lvl_off[c] + ((size_t)by * info->comp_bw[c] + bx) * 64 : NULL;
      /* DC */
      int s = huff_decode(&br, &dct[info->comp_td[c]]);
      if (s < 0 || s > 15) return JO_ERR_BAD_HUFFMAN;
      int diff = s ? extend(br_get(&br, s), s) : 0;
      pred[c] += diff;
      last_dc[c] = (uint32_t)diff * (uint32_t)q[0] + last_dc[c];
      blk[0] = clip16((int32_t)last_dc[c]);
      if (lv) lv[0] = (int16_t)pred[c];
      /* AC */
      const huff_t* ah = &act[info->comp_ta[c]];
      for (int k = 1; k < 64;) {
        int rs = huff_decode(&br, ah);
        if (rs < 0) return JO_ERR_BAD_HUFFMAN;
        int r = rs >> 4;
        s = rs & 15;
        if (s == 0) {
          if (r == 15) {
            k += 16;
            continue;
          }
          if (r != 0) return JO_ERR_BAD_HUFFMAN;
          break; /* EOB */
        }
        k += r;
        if (k > 63) return JO_ERR_BAD_HUFFMAN;
        int v = extend(br_get(&br, s), s);
        blk[kNatural[k]] = (int16_t)(v * (int)q[k]);
        if (lv) lv[kNatural[k]] = (int16_t)v;
        k++;
      }
    }
  }
  if (br.used_bits > br.real_bits) return JO_ERR_TRUNCATED;
  return JO_OK;
}

/* ------------------------------------------------------------------------ */
/* IDCTs                                                                     */
/* ------------------------------------------------------------------------ */

/* FFmpeg simple_idct, 8-bit (libavcodec/simple_idct_template.c, BIT_DEPTH 8,
 * extra_shift 0): W_i = round(cos(i*pi/16)*sqrt(2)*2^14), ROW_SHIFT 11,
 * COL_SHIFT 20, DC-only row shortcut (row[0] << 3, kept as int16).  The
 * "SUINT" arithmetic is emulated with uint32 and an int cast before the
 * arithmetic shift. */
#define SW1 22725
#define SW2 21407
#define SW3 19266
#define SW4 16383
#define SW5 12873
#define SW6 8867
#define SW7 4520
#define SROW_SHIFT 11
#define SCOL_SHIFT 20

static void simple_row(int16_t* row) {
  if (!(row[1] | row[2] | row[3] | row[4] | row[5] | row[6] | row[7])) {
    int16_t t = (int16_t)(uint16_t)((uint32_t)(int32_t)row[0] << 3);
    for (int i = 0; i < 8; i++) row[i] = t;
    return;
  }
  uint32_t a0, a1, a2, a3, b0, b1, b2, b3;
  a0 = (uint32_t)SW4 * (uint32_t)(int32_t)row[0] + (1u << (SROW_SHIFT - 1));
  a1 = a0;
  a2 = a0;
  a3 = a0;
  a0 += (uint32_t)SW2 * (uint32_t)(int32_t)row[2];
  a1 += (uint32_t)SW6 * (uint32_t)(int32_t)row[2];
  a2 -= (uint32_t)SW6 * (uint32_t)(int32_t)row[2];
  a3 -= (uint32_t)SW2 * (uint32_t)(int32_t)row[2];

  b0 = (uint32_t)(SW1 * row[1]);
  b0 += (uint32_t)SW3 * (uint32_t)(int32_t)row[3];
  b1 = (uint32_t)(SW3 * row[1]);
  b1 += (uint32_t)(-SW7) * (uint32_t)(int32_t)row[3];
  b2 = (uint32_t)(SW5 * row[1]);
  b2 += (uint32_t)(-SW1) * (uint32_t)(int32_t)row[3];
  b3 = (uint32_t)(SW7 * row[1]);
  b3 += (uint32_t)(-SW5) * (uint32_t)(int32_t)row[3];

  if (row[4] | row[5] | row[6] | row[7]) {
    a0 += (uint32_t)SW4 * (uint32_t)(int32_t)row[4] + (uint32_t)SW6 * (uint32_t)(int32_t)row[6];
    a1 += (uint32_t)(-SW4) * (uint32_t)(int32_t)row[4] - (uint32_t)SW2 * (uint32_t)(int32_t)row[6];
    a2 += (uint32_t)(-SW4) * (uint32_t)(int32_t)row[4] + (uint32_t)SW2 * (uint32_t)(int32_t)row[6];
    a3 += (uint32_t)SW4 * (uint32_t)(int32_t)row[4] - (uint32_t)SW6 * (uint32_t)(int32_t)row[6];
    b0 += (uint32_t)SW5 * (uint32_t)(int32_t)row[5];
    b0 += (uint32_t)SW7 * (uint32_t)(int32_t)row[7];
    b1 += (uint32_t)(-SW1) * (uint32_t)(int32_t)row[5];
    b1 += (uint32_t)(-SW5) * (uint32_t)(int32_t)row[7];
    b2 += (uint32_t)SW7 * (uint32_t)(int32_t)row[5];
    b2 += (uint32_t)SW3 * (uint32_t)(int32_t)row[7];
    b3 += (uint32_t)SW3 * (uint32_t)(int32_t)row[5];
    b3 += (uint32_t)(-SW1) * (uint32_t)(int32_t)row[7];
  }
  row[0] = (int16_t)((int32_t)(a0 + b0) >> SROW_SHIFT);
  row[7] = (int16_t)((int32_t)(a0 - b0) >> SROW_SHIFT);
  row[1] = (int16_t)((int32_t)(a1 + b1) >> SROW_SHIFT);
  row[6] = (int16_t)((int32_t)(a1 - b1) >> SROW_SHIFT);
  row[2] = (int16_t)((int32_t)(a2 + b2) >> SROW_SHIFT);
  row[5] = (int16_t)((int32_t)(a2 - b2) >> SROW_SHIFT);
  row[3] = (int16_t)((int32_t)(a3 + b3) >> SROW_SHIFT);
  row[4] = (int16_t)((int32_t)(a3 - b3) >> SROW_SHIFT);
}

static inline uint8_t clip_u8(int32_t v) { return v < 0 ? 0 : v > 255 ? 255 : (uint8_t)v; }

static void simple_col_put(uint8_t* dst, int stride, const int16_t* col) {
  uint32_t a0, a1, a2, a3, b0, b1, b2, b3;
  a0 = (uint32_t)SW4 * (uint32_t)(col[8 * 0] + ((1 << (SCOL_SHIFT - 1)) / SW4));
  a1 = a0;
  a2 = a0;
  a3 = a0;
  a0 += (uint32_t)SW2 * (uint32_t)(int32_t)col[8 * 2];
  a1 += (uint32_t)SW6 * (uint32_t)(int32_t)col[8 * 2];
  a2 += (uint32_t)(-SW6) * (uint32_t)(int32_t)col[8 * 2];
  a3 += (uint32_t)(-SW2) * (uint32_t)(int32_t)col[8 * 2];
  b0 = (uint32_t)(SW1 * col[8 * 1]);
  b1 = (uint32_t)(SW3 * col[8 * 1]);
  b2 = (uint32_t)(SW5 * col[8 * 1]);
  b3 = (uint32_t)(SW7 * col[8 * 1]);
  b0 += (uint32_t)SW3 * (uint32_t)(int32_t)col[8 * 3];
  b1 += (uint32_t)(-SW7) * (uint32_t)(int32_t)col[8 * 3];
  b2 += (uint32_t)(-SW1) * (uint32_t)(int32_t)col[8 * 3];
  b3 += (uint32_t)(-SW5) * (uint32_t)(int32_t)col[8 * 3];
  /* the sparse "if (col[8*k])" tests in FFmpeg only skip additions of zero */
  a0 += (uint32_t)SW4 * (uint32_t)(int32_t)col[8 * 4];
  a1 += (uint32_t)(-SW4) * (uint32_t)(int32_t)col[8 * 4];
  a2 += (uint32_t)(-SW4) * (uint32_t)(int32_t)col[8 * 4];
  a3 += (uint32_t)SW4 * (uint32_t)(int32_t)col[8 * 4];
  b0 += (uint32_t)SW5 * (uint32_t)(int32_t)col[8 * 5];
  b1 += (uint32_t)(-SW1) * (uint32_t)(int32_t)col[8 * 5];
  b2 += (uint32_t)SW7 * (uint32_t)(int32_t)col[8 * 5];
  b3 += (uint32_t)SW3 * (uint32_t)(int32_t)col[8 * 5];
  a0 += (uint32_t)SW6 * (uint32_t)(int32_t)col[8 * 6];
  a1 += (uint32_t)(-SW2) * (uint32_t)(int32_t)col[8 * 6];
  a2 += (uint32_t)SW2 * (uint32_t)(int32_t)col[8 * 6];
  a3 += (uint32_t)(-SW6) * (uint32_t)(int32_t)col[8 * 6];
  b0 += (uint32_t)SW7 * (uint32_t)(int32_t)col[8 * 7];
  b1 += (uint32_t)(-SW5) * (uint32_t)(int32_t)col[8 * 7];
  b2 += (uint32_t)SW3 * (uint32_t)(int32_t)col[8 * 7];
  b3 += (uint32_t)(-SW1) * (uint32_t)(int32_t)col[8 * 7];
  dst[0 * stride] = clip_u8((int32_t)(a0 + b0) >> SCOL_SHIFT);
  dst[1 * stride] = clip_u8((int32_t)(a1 + b1) >> SCOL_SHIFT);
  dst[2 * stride] = clip_u8((int32_t)(a2 + b2) >> SCOL_SHIFT);
  dst[3 * stride] = clip_u8((int32_t)(a3 + b3) >> SCOL_SHIFT);
  dst[4 * stride] = clip_u8((int32_t)(a3 - b3) >> SCOL_SHIFT);
  dst[5 * stride] = clip_u8((int32_t)(a2 - b2) >> SCOL_SHIFT);
  dst[6 * stride] = clip_u8((int32_t)(a1 - b1) >> SCOL_SHIFT);
  dst[7 * stride] = clip_u8((int32_t)(a0 - b0) >> SCOL_SHIFT);
}

void jo_idct_simple(const int16_t* in, uint8_t* out, int stride) {
  int16_t blk[64];
  memcpy(blk, in, sizeof(blk));
  for (int i = 0; i < 8; i++) simple_row(blk + 8 * i);
  for (int i = 0; i < 8; i++) simple_col_put(out + i, stride, blk + i);
}

/* IJG jidctint.c jpeg_idct_islow (libjpeg 9): CONST_BITS 13, PASS1_BITS 2,
 * columns first, zero-AC shortcuts in both passes (exact), output through the
 * range-limit table: sample = limit[(x >> 18) & 1023] with the range centre
 * (512 << 5) folded into the row-pass DC term. */
#define CB 13
#define P1 2
#define F0298 2446
#define F0390 3196
#define F0541 4433
#define F0765 6270
#define F0899 7373
#define F1175 9633
#define F1501 12299
#define F1847 15137
#define F1961 16069
#define F2053 16819
#define F2562 20995
#define F3072 25172

static inline uint8_t islow_limit(int32_t x) {
  int t = (int)(x & 1023); /* index into IDCT_range_limit */
  int v = t - 384;         /* sample_range_limit index */
  return v < 0 ? 0 : v > 255 ? 255 : (uint8_t)v;
}

void jo_idct_islow(const int16_t* in_biased, uint8_t* out, int stride) {
  /* coefficients carry FFmpeg's DC bias (1024); libjpeg's DC does not */
  int16_t in[64];
  memcpy(in, in_biased, sizeof(in));
  in[0] = (int16_t)(in[0] - JO_DC_BIAS);
  int32_t ws[64];
  for (int c = 0; c < 8; c++) {
    const int16_t* p = in + c;
    if (!(p[8] | p[16] | p[24] | p[32] | p[40] | p[48] | p[56])) {
      int32_t dc = (int32_t)p[0] * (1 << P1);
      for (int r = 0; r < 8; r++) ws[r * 8 + c] = dc;
      continue;
    }
    int32_t z1, z2, z3, t0, t1, t2, t3, t10, t11, t12, t13;
    z2 = p[0];
    z3 = p[32];
    z2 *= (1 << CB);
    z3 *= (1 << CB);
    z2 += 1 << (CB - P1 - 1);
    t0 = z2 + z3;
    t1 = z2 - z3;
    z2 = p[16];
    z3 = p[48];
    z1 = (z2 + z3) * F0541;
    t2 = z1 + z2 * F0765;
    t3 = z1 - z3 * F1847;
    t10 = t0 + t2;
    t13 = t0 - t2;
    t11 = t1 + t3;
    t12 = t1 - t3;
    t0 = p[56];
    t1 = p[40];
    t2 = p[24];
    t3 = p[8];
    z2 = t0 + t2;
    z3 = t1 + t3;
    z1 = (z2 + z3) * F1175;
    z2 = z2 * -F1961;
    z3 = z3 * -F0390;
    z2 += z1;
    z3 += z1;
    z1 = (t0 + t3) * -F0899;
    t0 = t0 * F0298;
    t3 = t3 * F1501;
    t0 += z1 + z2;
    t3 += z1 + z3;
    z1 = (t1 + t2) * -F2562;
    t1 = t1 * F2053;
    t2 = t2 * F3072;
    t1 += z1 + z3;
    t2 += z1 + z2;
    ws[0 * 8 + c] = (t10 + t3) >> (CB - P1);
    ws[7 * 8 + c] = (t10 - t3) >> (CB - P1);
    ws[1 * 8 + c] = (t11 + t2) >> (CB - P1);
    ws[6 * 8 + c] = (t11 - t2) >> (CB - P1);
    ws[2 * 8 + c] = (t12 + t1) >> (CB - P1);
    ws[5 * 8 + c] = (t12 - t1) >> (CB - P1);
    ws[3 * 8 + c] = (t13 + t0) >> (CB - P1);
    ws[4 * 8 + c] = (t13 - t0) >> (CB - P1);
  }
  for (int r = 0; r < 8; r++) {
    const int32_t* w = ws + r * 8;
    uint8_t* o = out + r * stride;
    int32_t z1, z2, z3, t0, t1, t2, t3, t10, t11, t12, t13;
    z2 = w[0] + ((512 << (P1 + 3)) + (1 << (P1 + 2)));
    if (!(w[1] | w[2] | w[3] | w[4] | w[5] | w[6] | w[7])) {
      uint8_t v = islow_limit(z2 >> (P1 + 3));
      for (int i = 0; i < 8; i++) o[i] = v;
      continue;
    }
    z3 = w[4];
    t0 = (z2 + z3) * (1 << CB);
    t1 = (z2 - z3) * (1 << CB);
    z2 = w[2];
    z3 = w[6];
    z1 = (z2 + z3) * F0541;
    t2 = z1 + z2 * F0765;
    t3 = z1 - z3 * F1847;
    t10 = t0 + t2;
    t13 = t0 - t2;
    t11 = t1 + t3;
    t12 = t1 - t3;
    t0 = w[7];
    t1 = w[5];
    t2 = w[3];
    t3 = w[1];
    z2 = t0 + t2;
    z3 = t1 + t3;
    z1 = (z2 + z3) * F1175;
    z2 = z2 * -F1961;
    z3 = z3 * -F0390;
    z2 += z1;
    z3 += z1;
    z1 = (t0 + t3) * -F0899;
    t0 = t0 * F0298;
    t3 = t3 * F1501;
    t0 += z1 + z2;
    t3 += z1 + z3;
    z1 = (t1 + t2) * -F2562;
    t1 = t1 * F2053;
    t2 = t2 * F3072;
    t1 += z1 + z3;
    t2 += z1 + z2;
    const int sh = CB + P1 + 3;
    o[0] = islow_limit((t10 + t3) >> sh);
    o[7] = islow_limit((t10 - t3) >> sh);
    o[1] = islow_limit((t11 + t2) >> sh);
    o[6] = islow_limit((t11 - t2) >> sh);
    o[2] = islow_limit((t12 + t1) >> sh);
    o[5] = islow_limit((t12 - t1) >> sh);
    o[3] = islow_limit((t13 + t0) >> sh);
    o[4] = islow_limit((t13 - t0) >> sh);
  }
}

/* ------------------------------------------------------------------------ */
/* Planes, colour                                                            */
/* ------------------------------------------------------------------------ */

size_t jo_planes_size(const jo_info* info) {
  size_t t = 0;
  for (int c = 0; c < info->ncomp; c++) t += (size_t)info->comp_bw[c] * info->comp_bh[c] * 64;
  return t;
}

static void plane_ptrs(const jo_info* info, const uint8_t* planes, const uint8_t** p, int* stride) {
  size_t o = 0;
  for (int c = 0; c < info->ncomp; c++) {
    p[c] = planes + o;
    stride[c] = info->comp_bw[c] * 8;
    o += (size_t)info->comp_bw[c] * info->comp_bh[c] * 64;
  }
}

static int decode_planes_info(const uint8_t* d, size_t size, const jo_info* info, int idct,
                              uint8_t* planes) {
  int16_t* coefs = (int16_t*)scratch(0, (size_t)info->nblocks * 64 * sizeof(int16_t));
  if (!coefs) return JO_ERR_BAD_HEADER;
  int rc = jo_decode_coefs(d, size, info, coefs, NULL);
  if (rc) return rc;
  const uint8_t* pc[JO_MAX_COMP];
  int st[JO_MAX_COMP];
  plane_ptrs(info, planes, pc, st);
  int nmcu = info->mcux * info->mcuy;
  for (int mcu = 0; mcu < nmcu; mcu++) {
    int mx = mcu % info->mcux, my = mcu / info->mcux;
    for (int b = 0; b < info->bpm; b++) {
      int c = info->mcu_comp[b];
      int bx = info->ncomp == 1 ? mx : mx * info->comp_h[c] + info->mcu_dx[b];
      int by = info->ncomp == 1 ? my : my * info->comp_v[c] + info->mcu_dy[b];
      uint8_t* dst = (uint8_t*)pc[c] + (size_t)by * 8 * st[c] + (size_t)bx * 8;
      const int16_t* blk = coefs + ((size_t)mcu * info->bpm + b) * 64;
      if (idct == JO_IDCT_ISLOW)
        jo_idct_islow(blk, dst, st[c]);
      else
        jo_idct_simple(blk, dst, st[c]);
    }
  }
  return JO_OK;
}

/* FFmpeg mjpegdec's in-decoder conversion of 4-component frames (the end of
 * ff_mjpeg_decode_frame / receive_frame, as recalled; parity UNPINNED):
 *   Adobe transform 0, pix_fmt GBRAP -- inverted CMYK to RGB (no Adobe marker:
 *   YCbCr + K, jo_frame_color, left as transform 1):
 *     R = c k 257 >> 16, G = m k 257 >> 16, B = y k 257 >> 16
 *   transform 2, YUVA444P -- YCCK to YCbCr:
 *     Y = (255 - y) k 257 >> 16, Cb = ((128 - cb) k 257 >> 16) + 128, Cr likewise
 * (c, m, y / y, cb, cr = components 0..2, k = component 3).  Planes 0..2 are
 * rewritten in place; transform 1 leaves them (YCbCr + K, K dropped). */
void jo_cmyk_transform(const jo_info* info, uint8_t* planes) {
  if (info->color != JO_COLOR_CMYK && info->color != JO_COLOR_YCCK) return;
  const uint8_t* pc[JO_MAX_COMP];
  int st[JO_MAX_COMP];
  plane_ptrs(info, planes, pc, st);
  for (int y = 0; y < info->height; y++)
    for (int x = 0; x < info->width; x++) {
      uint8_t* p0 = (uint8_t*)pc[0] + (size_t)y * st[0] + x;
      uint8_t* p1 = (uint8_t*)pc[1] + (size_t)y * st[1] + x;
      uint8_t* p2 = (uint8_t*)pc[2] + (size_t)y * st[2] + x;
      const int k = pc[3][(size_t)y * st[3] + x];
      if (info->color == JO_COLOR_YCCK) {
        const int r = (255 - *p0) * k, g = (128 - *p1) * k, b = (128 - *p2) * k;
        *p0 = (uint8_t)((r * 257) >> 16);
        *p1 = (uint8_t)(((g * 257) >> 16) + 128);
        *p2 = (uint8_t)(((b * 257) >> 16) + 128);
      } else {
        *p0 = (uint8_t)((*p0 * k * 257) >> 16);
        *p1 = (uint8_t)((*p1 * k * 257) >> 16);
        *p2 = (uint8_t)((*p2 * k * 257) >> 16);
      }
    }
}

int jo_decode_planes(const uint8_t* d, size_t size, int idct, uint8_t* planes) {
  jo_info info;
  int rc = jo_parse(d, size, &info);
  if (rc) return rc;
  return decode_planes_info(d, size, &info, idct, planes);
}

/* JFIF YCbCr -> RGB, integer tables as IJG jdcolor.c / jdmerge.c
 * (SCALEBITS 16, FIX(x) = (int)(x * 65536 + 0.5)). */
#define SCB 16
#define FIXC(x) ((int32_t)((x) * (1L << SCB) + 0.5))
typedef struct {
  int32_t cr_r[256], cb_b[256], cr_g[256], cb_g[256];
} csc_t;

static void build_csc(csc_t* t) {
  for (int i = 0; i < 256; i++) {
    int32_t x = i - 128;
    t->cr_r[i] = (FIXC(1.402) * x + (1 << (SCB - 1))) >> SCB;
    t->cb_b[i] = (FIXC(1.772) * x + (1 << (SCB - 1))) >> SCB;
    t->cr_g[i] = -FIXC(0.714136286) * x;
    t->cb_g[i] = -FIXC(0.344136286) * x + (1 << (SCB - 1));
  }
}

static inline void csc_px(const csc_t* t, int y, int cb, int cr, uint8_t* rgb) {
  rgb[0] = clip_u8(y + t->cr_r[cr]);
  rgb[1] = clip_u8(y + ((t->cb_g[cb] + t->cr_g[cr]) >> SCB));
  rgb[2] = clip_u8(y + t->cb_b[cb]);
}

static void store_px(uint8_t* out, int fmt, int ow, int oh, int x, int y, const uint8_t* rgb) {
  int swap = (fmt == JO_FMT_BGR || fmt == JO_FMT_BGR24);
  uint8_t c0 = swap ? rgb[2] : rgb[0], c1 = rgb[1], c2 = swap ? rgb[0] : rgb[2];
  if (fmt == JO_FMT_RGB || fmt == JO_FMT_BGR) {
    size_t pl = (size_t)ow * oh, o = (size_t)y * ow + x;
    out[o] = c0;
    out[pl + o] = c1;
    out[2 * pl + o] = c2;
  } else {
    size_t o = ((size_t)y * ow + x) * 3;
    out[o] = c0;
    out[o + 1] = c1;
    out[o + 2] = c2;
  }
}

static int planes_to_rgb(const jo_info* info, const uint8_t* planes, int fmt, uint8_t* out) {
  /* libjpeg's conversion to RGB (jdcolor.c): YCbCr, gray, and RGB-coded
   * frames (a copy); it has none for CMYK / YCCK */
  if (info->color != JO_COLOR_YCBCR && info->color != JO_COLOR_GRAY && info->color != JO_COLOR_RGB)
    return JO_ERR_UNSUPPORTED;
  const uint8_t* pc[JO_MAX_COMP];
  int st[JO_MAX_COMP];
  plane_ptrs(info, planes, pc, st);
  csc_t t;
  build_csc(&t);
  int W = info->width, H = info->height;
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) {
      uint8_t rgb[3];
      int yv = pc[0][(size_t)y * st[0] + x];
      if (info->ncomp == 1) {
        rgb[0] = rgb[1] = rgb[2] = (uint8_t)yv;
      } else if (info->color == JO_COLOR_RGB) { /* all components 1x1 */
        rgb[0] = (uint8_t)yv;
        rgb[1] = pc[1][(size_t)y * st[1] + x];
        rgb[2] = pc[2][(size_t)y * st[2] + x];
      } else {
        int cx1 = x * info->comp_h[1] / info->hmax, cy1 = y * info->comp_v[1] / info->vmax;
        int cx2 = x * info->comp_h[2] / info->hmax, cy2 = y * info->comp_v[2] / info->vmax;
        int cb = pc[1][(size_t)cy1 * st[1] + cx1];
        int cr = pc[2][(size_t)cy2 * st[2] + cx2];
        csc_px(&t, yv, cb, cr, rgb);
      }
      store_px(out, fmt, W, H, x, y, rgb);
    }
  return JO_OK;
}

/* chroma subsampling shifts of a 3-component frame (the yuvj4xxp format
 * FFmpeg's mjpeg decoder outputs: 444 / 422 / 420 / 440 / 411 ...) */
static int chroma_shifts(const jo_info* info, int* hsub, int* vsub) {
  *hsub = *vsub = 0;
  if (info->ncomp == 1) return JO_OK;
  if (info->comp_h[0] != info->hmax || info->comp_v[0] != info->vmax ||
      info->comp_h[1] != info->comp_h[2] || info->comp_v[1] != info->comp_v[2])
    return JO_ERR_UNSUPPORTED;
  int rh = info->hmax / info->comp_h[1], rv = info->vmax / info->comp_v[1];
  if (rh * info->comp_h[1] != info->hmax || rv * info->comp_v[1] != info->vmax) return JO_ERR_UNSUPPORTED;
  if ((rh & (rh - 1)) || (rv & (rv - 1)) || rh > 4 || rv > 4) return JO_ERR_UNSUPPORTED;
  while ((1 << *hsub) < rh) (*hsub)++;
  while ((1 << *vsub) < rv) (*vsub)++;
  return JO_OK;
}

/* swscale the decoded planes to sw x sh rgb24 (scratch slot 7). */
static int sws_planes(const jo_info* info, const uint8_t* planes, int sw, int sh, int filter,
                      uint8_t** rgb_out) {
  int hsub, vsub;
  int rc = chroma_shifts(info, &hsub, &vsub);
  if (rc) return rc;
  const uint8_t* pc[JO_MAX_COMP];
  int st[JO_MAX_COMP];
  plane_ptrs(info, planes, pc, st);
  jo_sws s;
  /* RGB planes (an RGB frame, or CMYK after the K transform) through the
   * luma filters; YCCK (after the transform) and YCbCr + K are YCbCr 4:4:4 */
  const int gbr = info->color == JO_COLOR_RGB || info->color == JO_COLOR_CMYK;
  if (jo_sws_init(&s, info->width, info->height, hsub, vsub, info->ncomp == 1 || gbr, sw, sh,
                  filter)) {
    jo_sws_free(&s);
    return JO_ERR_BAD_GEOMETRY;
  }
  s.gbr = gbr;
  uint8_t* rgb = (uint8_t*)scratch(7, (size_t)sw * sh * 3);
  rc = rgb ? jo_sws_scale(&s, pc, st, rgb) : -1;
  jo_sws_free(&s);
  if (rc) return JO_ERR_BAD_GEOMETRY;
  *rgb_out = rgb;
  return JO_OK;
}

int jo_decode_rgb_csc(const uint8_t* d, size_t size, int idct, int csc, int fmt, uint8_t* out) {
  jo_info info;
  int rc = jo_parse(d, size, &info);
  if (rc) return rc;
  uint8_t* planes = (uint8_t*)scratch(1, jo_planes_size(&info));
  if (!planes) return JO_ERR_BAD_HEADER;
  rc = decode_planes_info(d, size, &info, idct, planes);
  if (rc) return rc;
  if (csc == JO_CSC_JFIF) return planes_to_rgb(&info, planes, fmt, out);
  jo_cmyk_transform(&info, planes);
  uint8_t* rgb;
  rc = sws_planes(&info, planes, info.width, info.height, JO_FILTER_BICUBIC, &rgb);
  if (rc) return rc;
  const int W = info.width, H = info.height;
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) store_px(out, fmt, W, H, x, y, rgb + ((size_t)y * W + x) * 3);
  return JO_OK;
}

int jo_decode_rgb(const uint8_t* d, size_t size, int idct, int fmt, uint8_t* out) {
  return jo_decode_rgb_csc(d, size, idct, JO_CSC_SWSCALE, fmt, out);
}

int jo_sws_axis(int src, int dst, int kind, int align, int one, int src_pos, int dst_pos,
                int32_t* pos, int16_t* coef, int cap) {
  if (src <= 0 || dst <= 0) return -1;
  const int64_t inc = (((int64_t)src << 16) + (dst >> 1)) / dst;
  jo_sws_filter f;
  if (jo_sws_init_filter((int)inc, src, dst, align, one, kind, src_pos, dst_pos, &f)) return -1;
  int size = f.size;
  if ((int64_t)size * dst > cap) {
    jo_sws_filter_free(&f);
    return -1;
  }
  memcpy(pos, f.pos, sizeof(int32_t) * dst);
  memcpy(coef, f.coef, sizeof(int16_t) * (size_t)size * dst);
  jo_sws_filter_free(&f);
  return size;
}

/* ------------------------------------------------------------------------ */
/* Resize geometry (FFmpeg scale_eval.c ff_scale_adjust_dimensions semantics: */
/* av_rescale rounds to nearest; vf_pad x=-1 -> (W-w)/2; vf_crop centre).     */
/* ------------------------------------------------------------------------ */

static int64_t rescale_rnd(int64_t a, int64_t b, int64_t c) { return (a * b + c / 2) / c; }

int jo_geometry(int w, int h, const jo_resize* rs, jo_geom* g) {
  if (w <= 0 || h <= 0) return JO_ERR_BAD_GEOMETRY;
  int64_t fw = rs->fit_w > 0 ? rs->fit_w : w;
  int64_t fh = rs->fit_h > 0 ? rs->fit_h : h;
  int64_t sw = fw, sh = fh;
  if (rs->aspect != JO_ASPECT_NONE) {
    int64_t tw = rescale_rnd(fh, w, h), th = rescale_rnd(fw, h, w);
    if (rs->aspect == JO_ASPECT_DECREASE) {
      sw = tw < fw ? tw : fw;
      sh = th < fh ? th : fh;
    } else {
      sw = tw > fw ? tw : fw;
      sh = th > fh ? th : fh;
    }
  }
  if (sw < 1) sw = 1;
  if (sh < 1) sh = 1;
  int64_t cw = sw, ch = sh, px = 0, py = 0;
  if (rs->pad_w > 0 && rs->pad_h > 0) {
    cw = rs->pad_w;
    ch = rs->pad_h;
    if (cw < sw || ch < sh) return JO_ERR_BAD_GEOMETRY;
    px = (cw - sw) / 2;
    py = (ch - sh) / 2;
  }
  int64_t ow = cw, oh = ch, cx = 0, cy = 0;
  if (rs->crop_w > 0 && rs->crop_h > 0) {
    ow = rs->crop_w;
    oh = rs->crop_h;
    if (ow > cw || oh > ch) return JO_ERR_BAD_GEOMETRY;
    cx = (cw - ow) / 2;
    cy = (ch - oh) / 2;
  }
  if (sw > 65535 || sh > 65535 || ow > 65535 || oh > 65535) return JO_ERR_BAD_GEOMETRY;
  g->sw = (int)sw;
  g->sh = (int)sh;
  g->dx = (int)(px - cx);
  g->dy = (int)(py - cy);
  g->ow = (int)ow;
  g->oh = (int)oh;
  return JO_OK;
}

uint16_t jo_f32_to_f16(float f) {
  uint32_t x;
  memcpy(&x, &f, 4);
  uint32_t sign = (x >> 16) & 0x8000;
  uint32_t exp = (x >> 23) & 0xFF;
  uint32_t man = x & 0x7FFFFF;
  if (exp == 0xFF) return (uint16_t)(sign | 0x7C00 | (man ? 0x200 : 0));
  int e = (int)exp - 127 + 15;
  if (e >= 31) return (uint16_t)(sign | 0x7C00);
  if (e <= 0) {
    if (e < -10) return (uint16_t)sign;
    man |= 0x800000;
    int shift = 14 - e;
    uint32_t h = man >> shift;
    uint32_t rem = man & ((1u << shift) - 1), half = 1u << (shift - 1);
    if (rem > half || (rem == half && (h & 1))) h++;
    return (uint16_t)(sign | h);
  }
  uint32_t h = ((uint32_t)e << 10) | (man >> 13);
  uint32_t rem = man & 0x1FFF;
  if (rem > 0x1000 || (rem == 0x1000 && (h & 1))) h++;
  return (uint16_t)(sign | h);
}

/* fp32 -> bfloat16, round to nearest even (torch's Tensor.to(torch.bfloat16),
 * used after the reference's fp32 normalisation,
 * examples/imagenet_classification.py:95-106,162-163); NaN stays quiet NaN. */
uint16_t jo_f32_to_bf16(float f) {
  uint32_t x;
  memcpy(&x, &f, 4);
  if ((x & 0x7FFFFFFFu) > 0x7F800000u) return (uint16_t)((x >> 16) | 0x40);
  x += 0x7FFFu + ((x >> 16) & 1u);
  return (uint16_t)(x >> 16);
}

int jo_resize_planes(const jo_info* info, const uint8_t* planes, const jo_resize* rs, int fmt,
                     int dtype, const float* mean, const float* stdv, void* out,
                     jo_geom* geom_out) {
  jo_geom g;
  int rc = jo_geometry(info->width, info->height, rs, &g);
  if (rc) return rc;
  if (geom_out) *geom_out = g;
  /* one swscale pass to the scaled size (scale filter with rgb24 output),
   * then pad (black) / crop move pixels */
  uint8_t* rgbs;
  rc = sws_planes(info, planes, g.sw, g.sh, rs->filter, &rgbs);
  if (rc) return rc;
  int planar = (fmt == JO_FMT_RGB || fmt == JO_FMT_BGR);
  int swap = (fmt == JO_FMT_BGR || fmt == JO_FMT_BGR24);
  size_t pl = (size_t)g.ow * g.oh;
  for (int y = 0; y < g.oh; y++)
    for (int x = 0; x < g.ow; x++) {
      int cx = x - g.dx, cy = y - g.dy;
      uint8_t rgb[3] = {0, 0, 0};
      if (cx >= 0 && cx < g.sw && cy >= 0 && cy < g.sh) {
        const uint8_t* p = rgbs + ((size_t)cy * g.sw + cx) * 3;
        rgb[0] = p[0];
        rgb[1] = p[1];
        rgb[2] = p[2];
      }
      for (int ch = 0; ch < 3; ch++) {
        int src_ch = swap ? 2 - ch : ch;
        size_t oi = planar ? (size_t)ch * pl + (size_t)y * g.ow + x : ((size_t)y * g.ow + x) * 3 + ch;
        if (dtype == JO_DTYPE_U8) {
          ((uint8_t*)out)[oi] = rgb[src_ch];
        } else {
          float v = (float)rgb[src_ch] / 255.0f;
          v = v - mean[ch];
          v = v / stdv[ch];
          ((uint16_t*)out)[oi] = dtype == JO_DTYPE_BF16 ? jo_f32_to_bf16(v) : jo_f32_to_f16(v);
        }
      }
    }
  return JO_OK;
}

int jo_decode_resize(const uint8_t* d, size_t size, int idct, const jo_resize* rs, int fmt,
                     int dtype, const float* mean, const float* stdv, void* out,
                     jo_geom* geom_out) {
  jo_info info;
  int rc = jo_parse(d, size, &info);
  if (rc) return rc;
  uint8_t* planes = (uint8_t*)scratch(1, jo_planes_size(&info));
  if (!planes) return JO_ERR_BAD_HEADER;
  rc = decode_planes_info(d, size, &info, idct, planes);
  if (!rc) jo_cmyk_transform(&info, planes);
  if (!rc) rc = jo_resize_planes(&info, planes, rs, fmt, dtype, mean, stdv, out, geom_out);
  return rc;
}

/* ------------------------------------------------------------------------ */
/* Threaded batch drivers (CPU baseline: one decoder per thread, images     */
/* striped across threads, as examples/image_dataloading.py's workers).      */
/* ------------------------------------------------------------------------ */

typedef struct {
  const uint8_t* const* data;
  const size_t* sizes;
  int n, tid, nthreads, idct, fmt, dtype, resize;
  const jo_resize* rs;
  const float *mean, *stdv;
  uint8_t* out;
  size_t out_stride;
  int* status;
  int failed;
} job_t;

static void* worker(void* arg) {
  job_t* j = (job_t*)arg;
  for (int i = j->tid; i < j->n; i += j->nthreads) {
    int rc;
    if (j->resize)
      rc = jo_decode_resize(j->data[i], j->sizes[i], j->idct, j->rs, j->fmt, j->dtype, j->mean,
                            j->stdv, j->out + (size_t)i * j->out_stride, NULL);
    else
      rc = jo_decode_rgb(j->data[i], j->sizes[i], j->idct, j->fmt,
                         j->out + (size_t)i * j->out_stride);
    if (j->status) j->status[i] = rc;
    if (rc) j->failed++;
  }
  return NULL;
}

static int run_batch(job_t* proto, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  job_t jobs[256];
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = *proto;
    jobs[t].tid = t;
    jobs[t].nthreads = nthreads;
    jobs[t].failed = 0;
    if (nthreads > 1) pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  if (nthreads == 1) worker(&jobs[0]);
  int failed = 0;
  for (int t = 0; t < nthreads; t++) {
    if (nthreads > 1) pthread_join(th[t], NULL);
    failed += jobs[t].failed;
  }
  return failed;
}

int jo_decode_resize_batch(const uint8_t* const* data, const size_t* sizes, int n, int idct,
                           const jo_resize* rs, int fmt, int dtype, const float* mean,
                           const float* stdv, uint8_t* out, size_t out_stride, int nthreads,
                           int* status) {
  job_t j;
  memset(&j, 0, sizeof(j));
  j.data = data;
  j.sizes = sizes;
  j.n = n;
  j.idct = idct;
  j.fmt = fmt;
  j.dtype = dtype;
  j.resize = 1;
  j.rs = rs;
  j.mean = mean;
  j.stdv = stdv;
  j.out = out;
  j.out_stride = out_stride;
  j.status = status;
  return run_batch(&j, nthreads);
}

int jo_decode_rgb_batch(const uint8_t* const* data, const size_t* sizes, int n, int idct, int fmt,
                        uint8_t* out, size_t out_stride, int nthreads, int* status) {
  job_t j;
  memset(&j, 0, sizeof(j));
  j.data = data;
  j.sizes = sizes;
  j.n = n;
  j.idct = idct;
  j.fmt = fmt;
  j.out = out;
  j.out_stride = out_stride;
  j.status = status;
  return run_batch(&j, nthreads);
}

/* ---- NV12 -> planar RGB/BGR (the video path's colour conversion) ---------
 * Restates the reference kernel nv12_to_planar_rgb24
 * (src/libspdl/cuda/detail/color_conversion.cu:90-138, matrices :19-68,
 * wrapper src/libspdl/cuda/color_conversion.cpp:27-78): per 2x2 luma quad
 * one (U, V) pair; r = M[0][0]*(Y-16) + M[0][1]*(U-128) + M[0][2]*(V-128) in
 * fp32 with the multiply-adds contracted the way LLVM's DAG combiner fuses
 * (a*b + c*d) + e*f  ->  fma(e, f, fma(a, b, c*d)); clamp to [0, 255] and
 * truncate.  Quads with x + 1 >= width are not written (the reference
 * returns before writing them).  coeff outside 1..10 means 1 (BT.709).
 * Parity unpinned vs the CUDA build (no CUDA toolchain here): the
 * contraction order is the stated assumption. */
static const float jo_yuv2rgb[10][3][3] = {
    {{1.1644f, 0.0000f, 1.8337f}, {1.1644f, -0.2181f, -0.5451f}, {1.1644f, 2.1606f, 0.0000f}},
    {{1.1644f, 0.0000f, 1.8337f}, {1.1644f, -0.2181f, -0.5451f}, {1.1644f, 2.1606f, 0.0000f}},
    {{1.1644f, 0.0000f, 1.8337f}, {1.1644f, -0.2181f, -0.5451f}, {1.1644f, 2.1606f, 0.0000f}},
    {{1.1644f, 0.0000f, 1.6301f}, {1.1644f, -0.3864f, -0.8289f}, {1.1644f, 2.0726f, 0.0000f}},
    {{1.1644f, 0.0000f, 1.6325f}, {1.1644f, -0.4007f, -0.8315f}, {1.1644f, 2.0633f, 0.0000f}},
    {{1.1644f, 0.0000f, 1.6325f}, {1.1644f, -0.4007f, -0.8315f}, {1.1644f, 2.0633f, 0.0000f}},
    {{1.1644f, 0.0000f, 1.8351f}, {1.1644f, -0.2639f, -0.5550f}, {1.1644f, 2.1262f, 0.0000f}},
    {{1.1644f, 0.0000f, 1.8337f}, {1.1644f, -0.2181f, -0.5451f}, {1.1644f, 2.1606f, 0.0000f}},
    {{1.1689f, 0.0000f, 1.7237f}, {1.1689f, -0.1924f, -0.6679f}, {1.1689f, 2.1992f, 0.0000f}},
    {{1.1689f, 0.0000f, 1.7237f}, {1.1689f, -0.1924f, -0.6679f}, {1.1689f, 2.1992f, 0.0000f}},
};

static uint8_t jo_clamp8f(float x) { return x < 0.0f ? 0 : (x > 255.0f ? 255 : (uint8_t)x); }

void jo_nv12_to_rgb(const uint8_t* src, int frames, int height, int width, int bgr, int coeff,
                    uint8_t* dst) {
  if (coeff <= 0 || coeff > 10) coeff = 1;
  const float(*m)[3] = jo_yuv2rgb[coeff - 1];
  const size_t fsz = (size_t)(height + height / 2) * width, osz = (size_t)3 * height * width;
  for (int f = 0; f < frames; f++) {
    const uint8_t* yuv = src + f * fsz;
    uint8_t* rgb = dst + f * osz;
    for (int y = 0; y + 1 < height; y += 2)
      for (int x = 0; x + 1 < width; x += 2) {
        const uint8_t* uv = yuv + (size_t)(height + y / 2) * width + x;
        const float fu = (float)((int)uv[0] - 128), fv = (float)((int)uv[1] - 128);
        for (int dy = 0; dy < 2; dy++)
          for (int dx = 0; dx < 2; dx++) {
            const float fy = (float)((int)yuv[(size_t)(y + dy) * width + x + dx] - 16);
            for (int ch = 0; ch < 3; ch++) {
              const float v = fmaf(m[ch][2], fv, fmaf(m[ch][0], fy, m[ch][1] * fu));
              const int oc = bgr ? 2 - ch : ch;
              rgb[(size_t)oc * height * width + (size_t)(y + dy) * width + x + dx] = jo_clamp8f(v);
            }
          }
      }
  }
}
