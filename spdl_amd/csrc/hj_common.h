// hj_common.h -- layouts shared by the host driver and the gfx950 kernels.
//
// HBM layout of one batch (all offsets are per-image, computed on the host
// from the SOF probe, so every buffer is a flat allocation reused across
// batches):
//   bytes   : packed JPEG files, each at a 256-B aligned offset
//   clean   : destuffed entropy-coded bytes, same offsets as `bytes`
//   segs    : restart-segment start offsets (bytes into clean), seg_cap each
//   info    : ImageInfo (device parse result + status)
//   luts    : HuffTable[8] per image (DC0..3, AC0..3)
//   ents    : per block 64 u32 coefficient-list entries (BlockOut in
//             hj_kernels.hip); multiscan_kernel's int32 levels before that
//   bdesc   : per block {list start, count | DC << 16}
//   planes  : u8 component planes padded to whole blocks
//   wts     : swscale tables (positions, Q14/Q12 taps, row writers) per
//             distinct geometry of the batch (host-built, hj_sws.cpp)
#pragma once
#include <stdint.h>

#ifndef HJ_HD
#define HJ_HD __host__ __device__
#endif

namespace hj {

constexpr int kMaxComp = 4;  // 1 (gray), 3 (YCbCr / RGB) or 4 (Adobe CMYK / YCCK, all 1x1)

// The frame's colour model (spdl_hj_color), decided at the SOF as FFmpeg's
// mjpeg decoder picks the pix_fmt (oracle jo_frame_color): from the Adobe
// APP14 transform seen before the SOF (-1: none) and the component ids.
// false: a colour model this decoder does not take (RGB or 4-component
// frames with subsampled components).
enum { kColorGray = 0, kColorYcbcr, kColorRgb, kColorCmyk, kColorYcck, kColorYcbcrk };
inline HJ_HD bool frame_color(int ncomp, const int32_t* h, const int32_t* v, const int* ids,
                              int adobe, int32_t* color) {
  bool all11 = true;
  for (int c = 0; c < ncomp; c++) all11 = all11 && h[c] == 1 && v[c] == 1;
  if (ncomp == 1) {
    *color = kColorGray;
  } else if (ncomp == 3) {
    const bool rgb = adobe == 0 || (ids[0] == 'R' && ids[1] == 'G' && ids[2] == 'B');
    if (rgb && !all11) return false;
    *color = rgb ? kColorRgb : kColorYcbcr;
  } else {
    if (!all11) return false;
    *color = adobe == 0 ? kColorCmyk : adobe == 2 ? kColorYcck : kColorYcbcrk;
  }
  return true;
}
constexpr int kMaxBpm = 10;
constexpr int kLutBits = 10;
constexpr int kLutSize = 1 << kLutBits;
constexpr int kDcBias = 1024;  // FFmpeg mjpegdec last_dc start value (4 << bits)

// Parallel Huffman decode: a restart segment is cut into slots of N bits, at
// most kMaxSlots slots per pass; every slot keeps up to N + kRecPad symbol
// records (a symbol consumes >= 1 bit; +1 truncation marker; uint4 padding).
constexpr int kMaxSlots = 2048;
constexpr int kRecPad = 4;
constexpr int kMaxEntropyThreads = 1024;  // largest entropy workgroup

// Size-adaptive entropy decode: an image whose file holds more than the
// context's piece size (spdl_hj_set_param "entropy_piece_bytes") is decoded
// by P = ceil(bytes / piece) workgroups ("pieces"), at most kMaxPieces.
//  - with restart markers: piece p takes restart segments [p nseg / P,
//    (p + 1) nseg / P) -- independent, no hand-off;
//  - without: the P workgroups act as one workgroup of P x NT runs over the
//    one segment; the run-boundary states, block counts and DC sums cross
//    pieces through per-piece records of 8-byte {tag, value} granules
//    (EntChain) in the workspace's chain buffer, zeroed by parse_kernel.
// Work items (image | piece << 24) are handed out by a ticket counter, so a
// piece only ever waits for pieces of lower tickets, which are running.
constexpr int kMaxPieces = 64;
constexpr int kChainGranules = 16;  // per piece
constexpr int kChainHead = 32;      // granules before the first record (the ticket counter)
enum ChainSlot {
  kChG0 = 0, kChG1, kChL0, kChL1, kChT,  // rec1: first run's start state, last run's end state,
                                         // blocks started (the piece decoded from its own guess)
  kChE0, kChE1, kChB,                    // rec2: final end state, blocks through this piece
  kChDc = 8,                             // recDC: the piece's DC-difference sums, 4 components
};
enum ChainTag : uint32_t { kTagRec1 = 1, kTagRec2 = 2, kTagDc = 3, kTagFail = 0xFA11u };
// N for a scan whose longest segment has `maxbits` bits, at most `budget`
// slots per segment (kMaxSlots per workgroup decoding the segment)
inline HJ_HD uint32_t slot_bits(uint32_t maxbits, int sub_bits, uint32_t budget = kMaxSlots) {
  uint32_t need = (uint32_t)(((uint64_t)maxbits + budget - 1) / budget);
  need = (need + 31) & ~31u;
  const uint32_t n = (uint32_t)sub_bits;
  return need > n ? need : n;
}

// LUT entry (u32), everything a decode step needs precomputed:
//   [0,5)   bits the symbol takes: code + value bits (<= 16 + 15)
//   [5,7)   kind
//   [7,12)  value bits that follow the code (0 for Full)
//   [12,19) z advance: DC 1, AC coefficient run+1, ZRL 16, EOB or any other
//           size-0 AC symbol 64 (ends the block)
//   [19]    the symbol yields a coefficient
//   [20]    AC size-0 symbol other than EOB / ZRL (the sequential decoder
//           rejects it)
//   [21,32) Full: the value (int11); Sub: the sub-table index
constexpr uint32_t kKindSlow = 0;  // invalid, or a sub-table that did not fit
constexpr uint32_t kKindCode = 1;  // code resolved, value bits follow
constexpr uint32_t kKindFull = 2;  // code + value resolved
constexpr uint32_t kKindSub = 3;   // code longer than kLutBits: look up sub[idx][next 6 bits]
constexpr int kSubBits = 16 - kLutBits;
#ifndef HJ_SUB_POOL
#define HJ_SUB_POOL 2048
#endif
constexpr int kSubPool = HJ_SUB_POOL;  // entropy LDS entries for the second-level tables of a scan

// idct_rgb_kernel workgroup size: one block per thread, so a tile is
// kFusedThreads / bpm MCUs of one MCU row (host and kernel agree on it)
#ifndef HJ_FUSED_THREADS
#define HJ_FUSED_THREADS 256
#endif
constexpr int kFusedThreads = HJ_FUSED_THREADS;
constexpr int kMaxSub = 16;        // 64-entry sub-tables per Huffman table
constexpr int kEntHiShift = 21;    // value / sub-table index field

inline HJ_HD uint32_t hj_entry(uint32_t kind, int len, int sym, bool is_dc, int v) {
  const int size = is_dc ? sym : (sym & 15);
  const int run = is_dc ? 0 : (sym >> 4);
  uint32_t zinc, coef = 0, bad = 0;
  if (is_dc || size) {
    zinc = (uint32_t)run + 1u;
    coef = 1;
  } else if (run == 15) {
    zinc = 16;
  } else {
    zinc = 64;
    bad = run != 0;
  }
  const uint32_t sz = kind == kKindFull ? 0u : (uint32_t)size;
  return ((uint32_t)len + sz) | (kind << 5) | (sz << 7) | (zinc << 12) | (coef << 19) | (bad << 20) |
         (((uint32_t)v & 0x7FFu) << kEntHiShift);
}

struct HuffTable {
  uint32_t lut[kLutSize];
  uint32_t sub[kMaxSub << kSubBits];  // second level for codes of 11..16 bits
  int32_t nsub;
  int32_t long_slow;    // codes > kLutBits without sub-tables (canonical decode)
  int32_t sub_lo;       // the first level-1 index with a sub-table (its sub-table 0)
  int32_t maxcode[18];  // max code of length l (-1 if none), [17] sentinel
  int32_t valoff[17];
  uint8_t vals[256];
};

// The swscale conversion of one image (host plan, hj_sws.h): sizes, the
// offsets of its tables in the per-batch table pool (int32 units from
// ImageDesc::wt_off) and the sws_kernel tiling.
// packed_vscale's writer per output row (libswscale/output.c yuv2rgb_{X,2,1}_c
// and the _full_ variants), table entry: mode | yalpha << 4 | uvalpha << 17
enum { kSwsX = 0, kSwsOne = 1, kSwsTwo = 2 };
enum SwsTable { kHlPos = 0, kHlCoef, kHcPos, kHcCoef, kVlPos, kVlCoef, kVcPos, kVcCoef, kVmode, kSwsTables };
struct SwsDesc {
  int32_t sw, sh;          // scaled content size (the swscale destination)
  int32_t chr_w;           // chroma intermediate width (chrDstW)
  int32_t full, gray;      // SWS_FULL_CHR_H_INT; luma filters only (gray or gbr)
  int32_t hl_taps, hc_taps, vl_taps, vc_taps;  // taps read per output (trailing zeros cut)
  int32_t hl_size, hc_size, vl_size, vc_size;  // tap row stride (taps, multiple of 4)
  int32_t off[kSwsTables];
  int32_t rb;              // output rows per workgroup band
  int32_t col_chunk;       // output columns per workgroup
  int32_t gbr;             // three RGB planes (CMYK after the K transform), each
                           // through the luma filters (oracle sws_scale_gbr)
  // large downscale: the horizontal pass runs once per source row in
  // hscale_kernel (pre_rl luma / pre_rc chroma rows, row-major int16 in the
  // workspace's hbuf) and sws_kernel stages its bands from there
  int32_t pre, pre_rl, pre_rc;
};

struct ImageDesc {      // host-filled per image
  int64_t in_off;       // offset into bytes/clean
  int64_t in_size;
  int64_t coef_off;     // in blocks
  int64_t plane_off[kMaxComp];
  int64_t seg_off;      // entries into segs
  int64_t out_off;      // elements into the output
  int64_t wt_off;       // this image's swscale tables in the table pool (int32 units)
  int32_t seg_cap;
  int32_t width, height, ncomp;
  int32_t h_samp[kMaxComp], v_samp[kMaxComp];
  int32_t nblocks;
  int32_t plane_stride[kMaxComp];
  // output placement: out(x, y) = scaled(x - dx, y - dy), black outside
  int32_t dx, dy, ow, oh;
  SwsDesc sws;
  int64_t ds_off;       // destuff chunk records: offset and count
  int32_t ds_cap;
  int32_t color;        // spdl_hj_color (host probe)
  int64_t rec_off;      // entropy symbol records: offset (u32 units) and capacity
  int64_t rec_cap;
  int32_t pieces;       // entropy workgroups decoding this image (kMaxPieces)
  int32_t chain_off;    // its first piece record in the chain buffer (granules)
  // flat grids: the image's first workgroup in the destuff-chunk and IDCT
  // launches (one entry per workgroup in the dispatch maps, parse_kernel)
  int32_t ds_wg0, idct_wg0;
  int32_t hs_wg0, hs_wgs;  // hscale_kernel workgroups (SwsDesc::pre images)
  int32_t sws_wg0, sws_bands, sws_chunks;  // sws_kernel tiles: bands x column chunks
  int64_t hbuf_off;        // their horizontal-pass rows (int16 units)
};

// sws_kernel LDS budget per workgroup (bytes): the horizontal-pass columns of
// a band (int16 luma + two chroma planes), the u8 output tile and the band's
// vertical tables; the host picks the tallest band that fits.  32 KiB: the
// 2-lane schedule runs 3.6 % faster than at 48 KiB (smaller bands leave room
// for the other lane's workgroups; r02 A/B, 24 and 64 KiB slower)
#ifndef HJ_SWS_LDS_KB
#define HJ_SWS_LDS_KB 32
#endif
constexpr int kSwsLdsBudget = HJ_SWS_LDS_KB * 1024;
constexpr int kSwsMaxCols = 256;  // output columns per workgroup
// sws_kernel's LDS holds the horizontal pass column-major: a column of `rows`
// int16 samples (+ 4 slack rows read by zero taps) takes an odd number of
// words, so the 64 columns of a wave fall on distinct banks.  In int16 units.
inline HJ_HD int sws_col_stride(int rows) { return 2 * (((rows + 5) >> 1) | 1); }

struct ImageInfo {      // device-filled by the parse kernel
  int32_t status;
  int32_t width, height, ncomp, hmax, vmax, mcux, mcuy, bpm, nblocks, ri;
  int32_t scan_start;
  int32_t comp_h[kMaxComp], comp_v[kMaxComp];
  int32_t comp_bw[kMaxComp], comp_bh[kMaxComp];
  int32_t comp_w[kMaxComp], comp_hpx[kMaxComp];
  int32_t mcu_comp[kMaxBpm], mcu_dx[kMaxBpm], mcu_dy[kMaxBpm];
  int32_t dc_tab[kMaxComp], ac_tab[kMaxComp];  // table slot 0..7
  uint16_t qt[kMaxComp][64];                    // zig-zag order
  int32_t nseg;         // restart segments found by destuff
  int32_t clean_len;    // destuffed bytes
  int32_t sync_rounds;  // diagnostics: rounds the Huffman sync took
  int32_t scan_end;     // destuff: first byte past the entropy-coded data
  int32_t ent_wide;     // parse: the scan needs the entropy kernel's wide path (5-6 distinct
                        // tables, long codes outside the LDS sub-table pool or slow codes)
  int32_t multiscan;    // parse: progressive, or sequential with non-interleaved scans
                        // (multiscan_kernel decodes it; destuff / entropy skip it)
  int32_t progressive;  // parse: SOF2
  int32_t color;        // parse: spdl_hj_color, decided at the SOF (frame_color)
  // Huffman tables by slot (DC 0..3, AC 4..7): file offset of the DHT entry's 16
  // length bytes, number of symbols (0: absent), a hash of lengths + symbols
  // (parse), and the table (image * 8 + slot in the LUT pool) that lut_kernel
  // built for it -- the first image of the batch whose table has these bytes
  int32_t tab_off[8], tab_n[8];
  uint32_t tab_hash[8];
  int32_t lut_ref[8];
  int64_t tphase[4];    // diagnostics: wall_clock64 ticks of the entropy phases
  int64_t dbg[4];       // diagnostics: symbols (round 0), wave iterations, shader clocks, rt ticks
  int32_t sdiag[48];    // diagnostics, multiscan: per scan (16) start / end (wall_clock64
                        // ticks from the decode start) and Huffman symbols decoded
};

// destuff: chunk-parallel over kDsChunk-byte chunks; per-chunk counts and prefixes
constexpr int kDsChunk = 4096;
// idct_kernel: one block per thread, kIdctThreads blocks per workgroup
#ifndef HJ_IDCT_THREADS
#define HJ_IDCT_THREADS 256
#endif
constexpr int kIdctThreads = HJ_IDCT_THREADS;
// hscale_kernel: source rows of one plane per workgroup
constexpr int kHsRows = 16;
struct DsChunk {
  int32_t keep, rst, term;
  int32_t keep_pre, rst_pre;
  int32_t pad_[3];
};

struct BatchParams {
  int32_t n;
  int32_t pix_fmt, dtype, idct;
  int32_t resize, filter;
  int32_t out_w, out_h;  // full-res mode: common size
  int32_t sub_bits;      // Huffman subsequence size (bits, multiple of 32)
  int32_t debug_mask;    // diagnostics: skip kernel phases (timing ablations only)
  int32_t xcd_order;     // XCD-aware tile order ("xcd_order"): bit 0 sws_kernel, bit 1 idct_kernel
  float mean[3], std[3];
  // ff_yuv2rgb_c_init_tables coefficients (hj_sws.h SwsCsc)
  int32_t crv, cbu, cgu, cgv;
  int32_t y_coeff, y_offset, v2r, v2g, u2g, u2b;
};

enum Status {
  kOk = 0,
  kErrNotJpeg = 1,
  kErrUnsupported = 2,
  kErrBadHeader = 3,
  kErrBadHuffman = 4,
  kErrTruncated = 5,
  kErrBadRestart = 6,
  kErrBadGeometry = 7,
  kErrDevice = 9,    // SPDL_HJ_ERR_HIP
  kErrHandoff = 11,  // SPDL_HJ_ERR_HANDOFF: a piece hand-off wait gave up; the host re-decodes
                     // the image in one workgroup (spdl_hj_wait / collect_status)
};

}  // namespace hj
