/*
 * ljpin.c -- pins the oracle against IJG libjpeg 9d (/opt/conda/lib/libjpeg.so.9).
 *
 * TEST INFRASTRUCTURE ONLY: used by tests/gen_golden.py (and the pin tests
 * when the library is present) to produce independent golden vectors:
 *   - lj_read_coefs: quantised coefficients via jpeg_read_coefficients(), the
 *     entropy-decode + DC-prediction ground truth (natural order, per
 *     component, block rows padded to the sampling factor).
 *   - lj_decode_rgb: full decode with dct_method = JDCT_ISLOW and
 *     do_fancy_upsampling = FALSE (nearest chroma), out_color_space = JCS_RGB.
 * libjpeg is a third-party implementation of T.81, not SPDL; see DESIGN.md.
 */
#include <setjmp.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "jpeglib.h"

typedef struct {
  struct jpeg_error_mgr pub;
  jmp_buf jb;
} err_t;

static void on_error(j_common_ptr c) {
  err_t* e = (err_t*)c->err;
  longjmp(e->jb, 1);
}
static void on_message(j_common_ptr c, int lvl) { (void)c; (void)lvl; }

static void mem_src_init(j_decompress_ptr c) { (void)c; }
static boolean mem_fill(j_decompress_ptr c) {
  static const JOCTET eoi[2] = {0xFF, 0xD9};
  c->src->next_input_byte = eoi;
  c->src->bytes_in_buffer = 2;
  return TRUE;
}
static void mem_skip(j_decompress_ptr c, long n) {
  if (n <= 0) return;
  if ((size_t)n > c->src->bytes_in_buffer) n = (long)c->src->bytes_in_buffer;
  c->src->next_input_byte += n;
  c->src->bytes_in_buffer -= (size_t)n;
}
static void mem_term(j_decompress_ptr c) { (void)c; }

static void set_src(j_decompress_ptr c, struct jpeg_source_mgr* s, const uint8_t* d, size_t n) {
  s->init_source = mem_src_init;
  s->fill_input_buffer = mem_fill;
  s->skip_input_data = mem_skip;
  s->resync_to_restart = jpeg_resync_to_restart;
  s->term_source = mem_term;
  s->next_input_byte = d;
  s->bytes_in_buffer = n;
  c->src = s;
}

/* info[0..]: width, height, ncomp, then per comp: bw, bh, h, v ; qt: 4x64 natural */
int lj_read_coefs(const uint8_t* d, size_t n, int* info, int16_t* out, size_t out_cap,
                  uint16_t* qt) {
  struct jpeg_decompress_struct c;
  err_t e;
  struct jpeg_source_mgr src;
  c.err = jpeg_std_error(&e.pub);
  e.pub.error_exit = on_error;
  e.pub.emit_message = on_message;
  if (setjmp(e.jb)) {
    jpeg_destroy_decompress(&c);
    return -1;
  }
  jpeg_create_decompress(&c);
  set_src(&c, &src, d, n);
  jpeg_read_header(&c, TRUE);
  jvirt_barray_ptr* arr = jpeg_read_coefficients(&c);
  info[0] = (int)c.image_width;
  info[1] = (int)c.image_height;
  info[2] = c.num_components;
  size_t o = 0;
  for (int ci = 0; ci < c.num_components; ci++) {
    jpeg_component_info* cp = &c.comp_info[ci];
    int bw = (int)cp->width_in_blocks, bh = (int)cp->height_in_blocks;
    if (c.num_components > 1) {
      bw = (bw + cp->h_samp_factor - 1) / cp->h_samp_factor * cp->h_samp_factor;
      bh = (bh + cp->v_samp_factor - 1) / cp->v_samp_factor * cp->v_samp_factor;
    }
    info[3 + 4 * ci] = bw;
    info[4 + 4 * ci] = bh;
    info[5 + 4 * ci] = cp->h_samp_factor;
    info[6 + 4 * ci] = cp->v_samp_factor;
    for (int r = 0; r < bh; r++) {
      JBLOCKARRAY row = (*c.mem->access_virt_barray)((j_common_ptr)&c, arr[ci], (JDIMENSION)r, 1, FALSE);
      for (int b = 0; b < bw; b++) {
        if (o + 64 > out_cap) {
          jpeg_destroy_decompress(&c);
          return -2;
        }
        for (int k = 0; k < 64; k++) out[o + k] = row[0][b][k];
        o += 64;
      }
    }
    if (cp->quant_table && cp->quant_tbl_no < 4)
      for (int k = 0; k < 64; k++) qt[cp->quant_tbl_no * 64 + k] = cp->quant_table->quantval[k];
  }
  jpeg_finish_decompress(&c);
  jpeg_destroy_decompress(&c);
  return (int)(o / 64);
}

int lj_decode_rgb(const uint8_t* d, size_t n, uint8_t* out, size_t cap, int* w, int* h) {
  struct jpeg_decompress_struct c;
  err_t e;
  struct jpeg_source_mgr src;
  c.err = jpeg_std_error(&e.pub);
  e.pub.error_exit = on_error;
  e.pub.emit_message = on_message;
  if (setjmp(e.jb)) {
    jpeg_destroy_decompress(&c);
    return -1;
  }
  jpeg_create_decompress(&c);
  set_src(&c, &src, d, n);
  jpeg_read_header(&c, TRUE);
  c.out_color_space = JCS_RGB;
  c.dct_method = JDCT_ISLOW;
  c.do_fancy_upsampling = FALSE;
  c.do_block_smoothing = FALSE;
  jpeg_start_decompress(&c);
  *w = (int)c.output_width;
  *h = (int)c.output_height;
  size_t stride = (size_t)c.output_width * 3;
  if (stride * c.output_height > cap) {
    jpeg_destroy_decompress(&c);
    return -2;
  }
  while (c.output_scanline < c.output_height) {
    JSAMPROW row = out + stride * c.output_scanline;
    jpeg_read_scanlines(&c, &row, 1);
  }
  jpeg_finish_decompress(&c);
  jpeg_destroy_decompress(&c);
  return 0;
}

/* ---- fixture encoder: a sequential (SOF0) JPEG whose components are coded
 * in separate, non-interleaved scans (one scan per component, Ss=0 Se=63),
 * the multi-scan sequential layout Pillow cannot write.  rgb: h*w*ncomp
 * (ncomp 1 or 3), h_samp/v_samp of component 0 (chroma 1x1).  Returns the
 * JPEG size, or -1 / -(needed) when out_cap is too small. */
static void dst_init(j_compress_ptr c) { (void)c; }
static boolean dst_empty(j_compress_ptr c) { (void)c; return FALSE; }
static void dst_term(j_compress_ptr c) { (void)c; }

long lj_encode_multiscan(const uint8_t* px, int w, int h, int ncomp, int quality, int h0, int v0,
                         int restart_blocks, uint8_t* out, size_t out_cap) {
  struct jpeg_compress_struct c;
  err_t e;
  struct jpeg_destination_mgr dst;
  c.err = jpeg_std_error(&e.pub);
  e.pub.error_exit = on_error;
  e.pub.emit_message = on_message;
  if (setjmp(e.jb)) {
    jpeg_destroy_compress(&c);
    return -1;
  }
  jpeg_create_compress(&c);
  dst.init_destination = dst_init;
  dst.empty_output_buffer = dst_empty;
  dst.term_destination = dst_term;
  dst.next_output_byte = out;
  dst.free_in_buffer = out_cap;
  c.dest = &dst;
  c.image_width = (JDIMENSION)w;
  c.image_height = (JDIMENSION)h;
  c.input_components = ncomp;
  c.in_color_space = ncomp == 3 ? JCS_RGB : JCS_GRAYSCALE;
  jpeg_set_defaults(&c);
  jpeg_set_quality(&c, quality, TRUE);
  if (ncomp == 3) {
    c.comp_info[0].h_samp_factor = h0;
    c.comp_info[0].v_samp_factor = v0;
  }
  c.restart_in_rows = 0;
  c.restart_interval = (unsigned)restart_blocks;
  static jpeg_scan_info scans[3];
  for (int i = 0; i < ncomp; i++) {
    scans[i].comps_in_scan = 1;
    scans[i].component_index[0] = ncomp - 1 - i; /* reverse order: not the frame order */
    scans[i].Ss = 0;
    scans[i].Se = 63;
    scans[i].Ah = 0;
    scans[i].Al = 0;
  }
  c.scan_info = scans;
  c.num_scans = ncomp;
  jpeg_start_compress(&c, TRUE);
  while (c.next_scanline < c.image_height) {
    JSAMPROW row = (JSAMPROW)(px + (size_t)c.next_scanline * w * ncomp);
    jpeg_write_scanlines(&c, &row, 1);
  }
  jpeg_finish_compress(&c);
  long n = (long)(out_cap - dst.free_in_buffer);
  jpeg_destroy_compress(&c);
  return n;
}

/* Fixture encoder for the non-YCbCr colour spaces, every component 1x1:
 *   mode 0: 4-component CMYK from CMYK pixels (libjpeg's Adobe convention:
 *           the values are written as given, APP14 transform 0)
 *   mode 1: 4-component YCCK from CMYK pixels (APP14 transform 2)
 *   mode 2: 3-component RGB from RGB pixels (component ids 'R', 'G', 'B',
 *           APP14 transform 0, no colour transform)
 * plus the scan script: mode | 4 progressive (jpeg_simple_progression),
 * mode | 8 sequential with one component per scan (non-interleaved). */
long lj_encode_cs(const uint8_t* px, int w, int h, int quality, int mode, int restart_blocks,
                  uint8_t* out, size_t out_cap) {
  struct jpeg_compress_struct c;
  err_t e;
  struct jpeg_destination_mgr dst;
  c.err = jpeg_std_error(&e.pub);
  e.pub.error_exit = on_error;
  e.pub.emit_message = on_message;
  if (setjmp(e.jb)) {
    jpeg_destroy_compress(&c);
    return -1;
  }
  jpeg_create_compress(&c);
  dst.init_destination = dst_init;
  dst.empty_output_buffer = dst_empty;
  dst.term_destination = dst_term;
  dst.next_output_byte = out;
  dst.free_in_buffer = out_cap;
  c.dest = &dst;
  c.image_width = (JDIMENSION)w;
  c.image_height = (JDIMENSION)h;
  const int cs = mode & 3;
  const int nc = cs == 2 ? 3 : 4;
  c.input_components = nc;
  c.in_color_space = cs == 2 ? JCS_RGB : JCS_CMYK;
  jpeg_set_defaults(&c);
  jpeg_set_colorspace(&c, cs == 2 ? JCS_RGB : cs == 1 ? JCS_YCCK : JCS_CMYK);
  jpeg_set_quality(&c, quality, TRUE);
  for (int i = 0; i < nc; i++) c.comp_info[i].h_samp_factor = c.comp_info[i].v_samp_factor = 1;
  c.restart_interval = (unsigned)restart_blocks;
  static jpeg_scan_info seq[4];
  if (mode & 4) {
    jpeg_simple_progression(&c);
  } else if (mode & 8) {
    for (int i = 0; i < nc; i++) {
      seq[i].comps_in_scan = 1;
      seq[i].component_index[0] = i;
      seq[i].Ss = 0;
      seq[i].Se = 63;
      seq[i].Ah = 0;
      seq[i].Al = 0;
    }
    c.scan_info = seq;
    c.num_scans = nc;
  }
  jpeg_start_compress(&c, TRUE);
  while (c.next_scanline < c.image_height) {
    JSAMPROW row = (JSAMPROW)(px + (size_t)c.next_scanline * w * nc);
    jpeg_write_scanlines(&c, &row, 1);
  }
  jpeg_finish_compress(&c);
  long n = (long)(out_cap - dst.free_in_buffer);
  jpeg_destroy_compress(&c);
  return n;
}
