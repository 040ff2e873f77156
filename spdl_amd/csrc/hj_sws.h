// hj_sws.h -- host-side plan of the scale / colour-conversion stage.
//
// The reference's CPU path converts the decoded yuvj4xxp frame to rgb24 with
// ONE libswscale context (the scale filter of the graph SPDL builds,
// src/spdl/io/_preprocessing.py:214-254, run by FilterGraphImpl::filter,
// src/libspdl/core/detail/ffmpeg/filter_graph.cpp:280-313; pad/crop only move
// pixels afterwards).  Everything that context decides from the geometry alone
// -- filter taps and positions per axis, chroma sizes, the full-chroma switch,
// which output writer each row uses, the yuv2rgb coefficients -- is computed
// here on the host, once per distinct geometry, and shipped to the device as
// one int32 blob; the gfx950 kernel (sws_kernel) only runs the arithmetic.
#pragma once
#include <stdint.h>

#include <vector>

#include "hj_common.h"

namespace hj {

// One axis of libswscale's initFilter (utils.c): per output sample the first
// source sample and `size` taps normalised to `one`.
struct SwsAxis {
  int size = 0, n = 0;
  int eff = 0;  // taps actually non-zero at the end of some row (<= size)
  std::vector<int32_t> pos;
  std::vector<int16_t> coef;
};

struct SwsPlan {
  int srcW = 0, srcH = 0, dstW = 0, dstH = 0;
  int chrSrcW = 0, chrSrcH = 0, chrDstW = 0, chrDstH = 0;
  int hsub = 0, vsub = 0;  // source chroma subsampling shifts
  bool full = false;       // SWS_FULL_CHR_H_INT
  bool gray = false;
  bool special = false;    // unscaled yuv420p/422p -> rgb24 converter
  SwsAxis hl, hc, vl, vc;
  std::vector<int32_t> vmode;  // per output row
};

// Coefficients of ff_yuv2rgb_c_init_tables for a full-range BT.601 source.
struct SwsCsc {
  int32_t crv, cbu, cgu, cgv;                    // table increments (cy-scaled)
  int32_t y_coeff, y_offset, v2r, v2g, u2g, u2b;  // yuv2rgb_write_full
};
SwsCsc sws_csc();

// kind: SPDL_HJ_FILTER_*.  Returns 0, or an SPDL_HJ_ERR_* code (a filter
// longer than swscale handles without cascading: BAD_GEOMETRY).
int sws_plan(int srcW, int srcH, int hsub, int vsub, bool gray, int dstW, int dstH, int kind,
             SwsPlan* out);

}  // namespace hj
