// hj_sws.cpp -- host-side plan of the swscale conversion (see hj_sws.h).
//
// The algorithm is libswscale's (third-party FFmpeg, CI pin conda-forge
// ffmpeg 8.0, .github/workflows/_build_linux.yml:127), x86-64 build:
//   sws_init_context   (libswscale/utils.c)  chroma sizes, xInc, forced full
//                                            chroma, get_local_pos siting
//   initFilter         (utils.c)             taps per axis
//   packed_vscale      (vscale.c)            writer per output row
//   ff_yuv2rgb_c_init_tables (yuv2rgb.c)     BT.601 full-range coefficients
//   ff_get_unscaled_swscale                  yuv2rgb_c_24_rgb special case
// The test oracle restates the same algorithm separately
// (oracle/sws_oracle.c); the GPU parity tests compare the two end to end.
#include "hj_sws.h"

#include <math.h>
#include <string.h>

#include <algorithm>

#include "../../include/spdl_hipjpeg.h"

namespace hj {
namespace {

constexpr double kReduceCutoff = 0.002;  // SWS_MAX_REDUCE_CUTOFF
constexpr int kMaxFilterSize = 256;      // SWS_MAX_FILTER_SIZE (longer -> cascade)

inline int64_t c_div(int64_t a, int64_t b) { return a / b; }  // C: truncates
inline int64_t rounded_div(int64_t a, int64_t b) { return (a >= 0 ? a + (b >> 1) : a - (b >> 1)) / b; }
inline int ilog2(unsigned v) { return v ? 31 - __builtin_clz(v) : 0; }  // av_log2

// The fixed-point kernel value at distance d (2^30 = one source sample after
// the downscale widening) for swscale's SWS_BICUBIC / SWS_BILINEAR /
// SWS_LANCZOS, in units of `fone`.
int64_t kernel_tap(int kind, int64_t d, int64_t fone) {
  if (kind == SPDL_HJ_FILTER_BILINEAR) {
    int64_t c = (1 << 30) - d;
    return (c < 0 ? 0 : c) * (fone >> 30);
  }
  if (kind == SPDL_HJ_FILTER_LANCZOS) {
    const double p = 3.0, x = d * (1.0 / (1 << 30));
    int64_t c = (int64_t)((d ? sin(x * M_PI) * sin(x * M_PI / p) / (x * x * M_PI * M_PI / p) : 1.0) *
                          fone);
    return x > p ? 0 : c;
  }
  // Mitchell-Netravali with swscale's defaults B = 0, C = 0.6 in Q24
  const int64_t B = 0, C = (int64_t)(0.6 * (1 << 24));
  int64_t c = 0;
  if (d < 1LL << 31) {
    const int64_t d2 = (d * d) >> 30, d3 = (d2 * d) >> 30;
    if (d < 1LL << 30)
      c = (12 * (1 << 24) - 9 * B - 6 * C) * d3 + (-18 * (1 << 24) + 12 * B + 6 * C) * d2 +
          (6 * (1 << 24) - 2 * B) * (1 << 30);
    else
      c = (-B - 6 * C) * d3 + (6 * B + 30 * C) * d2 + (-12 * B - 48 * C) * d +
          (8 * B + 24 * C) * (1 << 30);
  }
  return c / ((1LL << 54) / fone);
}

class FilterBuilder {
 public:
  FilterBuilder(int xInc, int src, int dst, int align, int one, int kind, int src_pos, int dst_pos)
      : xinc_(xInc), src_(src), dst_(dst), align_(align), one_(one), kind_(kind), sp_(src_pos),
        dp_(dst_pos) {
    const int r = ilog2((unsigned)(src / dst));
    fone_ = 1LL << (54 - (r < 8 ? r : 8));
  }

  bool build(SwsAxis* out) {
    sample();
    const int fs = reduce();
    if (fs >= kMaxFilterSize) return false;
    fold_borders(fs);
    normalise(fs, out);
    return true;
  }

 private:
  // initial taps: identity when unscaled, else the kernel over a window of
  // `size_` samples starting at the truncated (C division) window origin
  void sample() {
    pos_.assign(dst_, 0);
    if (llabs((int64_t)xinc_ - 0x10000) < 10 && sp_ == dp_) {
      size_ = 1;
      taps_.assign(dst_, fone_);
      for (int i = 0; i < dst_; i++) pos_[i] = i;
      return;
    }
    const int factor = kind_ == SPDL_HJ_FILTER_BILINEAR ? 2 : kind_ == SPDL_HJ_FILTER_LANCZOS ? 6 : 4;
    size_ = xinc_ <= (1 << 16) ? 1 + factor : 1 + (factor * src_ + dst_ - 1) / dst_;
    size_ = std::max(1, std::min(size_, src_ - 2));
    taps_.assign((size_t)dst_ * size_, 0);
    int64_t center = ((dp_ * (int64_t)xinc_) >> 7) - ((sp_ * 0x10000LL) >> 7);  // Q17
    for (int i = 0; i < dst_; i++, center += 2LL * xinc_) {
      int xx = (int)c_div(center - (size_ - 2) * (1LL << 16), 1 << 17);
      pos_[i] = xx;
      for (int j = 0; j < size_; j++, xx++) {
        int64_t d = llabs((int64_t)xx * (1 << 17) - center) << 13;
        if (xinc_ > 1 << 16) d = d * dst_ / src_;
        taps_[(size_t)i * size_ + j] = kernel_tap(kind_, d, fone_);
      }
    }
  }

  // drop near-zero taps (cumulative |tap| <= 0.002) from the left of every
  // row while positions stay monotonic, measure the widest row's right
  // trim, align the size
  int reduce() {
    const double cut = kReduceCutoff * fone_;
    int widest = 0;
    for (int i = dst_ - 1; i >= 0; i--) {
      int64_t* row = &taps_[(size_t)i * size_];
      int64_t acc = 0;
      for (int j = 0; j < size_; j++) {
        acc += llabs(row[0]);
        if (acc > cut) break;
        if (i < dst_ - 1 && pos_[i] >= pos_[i + 1]) break;
        std::copy(row + 1, row + size_, row);
        row[size_ - 1] = 0;
        pos_[i]++;
      }
      int keep = size_;
      acc = 0;
      for (int j = size_ - 1; j > 0; j--) {
        acc += llabs(row[j]);
        if (acc > cut) break;
        keep--;
      }
      widest = std::max(widest, keep);
    }
    int align = align_;
    if (widest == 1 && align == 2) align = 1;  // x86: unscaled vertical stays 1
    const int fs = (widest + align - 1) & ~(align - 1);
    std::vector<int64_t> t((size_t)dst_ * fs, 0);
    for (int i = 0; i < dst_; i++)
      for (int j = 0; j < fs && j < size_; j++) t[(size_t)i * fs + j] = taps_[(size_t)i * size_ + j];
    taps_.swap(t);
    size_ = fs;
    return fs;
  }

  // taps left of sample 0 / right of src-1 fold into the edge sample
  void fold_borders(int fs) {
    for (int i = 0; i < dst_; i++) {
      int64_t* row = &taps_[(size_t)i * fs];
      if (pos_[i] < 0) {
        for (int j = 1; j < fs; j++) {
          const int to = std::max(j + pos_[i], 0);
          row[to] += row[j];
          row[j] = 0;
        }
        pos_[i] = 0;
      }
      if (pos_[i] + fs > src_) {
        const int shift = pos_[i] + std::min(fs - src_, 0);
        int64_t spill = 0;
        for (int j = fs - 1; j >= 0; j--)
          if (pos_[i] + j >= src_) {
            spill += row[j];
            row[j] = 0;
          }
        for (int j = fs - 1; j >= 0; j--) row[j] = j < shift ? 0 : row[j - shift];
        pos_[i] -= shift;
        row[src_ - 1 - pos_[i]] += spill;
      }
    }
  }

  void normalise(int fs, SwsAxis* out) {
    out->size = fs;
    out->n = dst_;
    out->pos = pos_;
    out->coef.assign((size_t)dst_ * fs, 0);
    out->eff = 1;
    for (int i = 0; i < dst_; i++) {
      const int64_t* row = &taps_[(size_t)i * fs];
      int64_t sum = 0, err = 0;
      for (int j = 0; j < fs; j++) sum += row[j];
      sum = (sum + one_ / 2) / one_;
      if (!sum) sum = 1;
      for (int j = 0; j < fs; j++) {
        const int64_t v = row[j] + err;
        const int q = (int)rounded_div(v, sum);
        out->coef[(size_t)i * fs + j] = (int16_t)q;
        err = v - (int64_t)q * sum;
        if (q) out->eff = std::max(out->eff, j + 1);
      }
    }
  }

  int xinc_, src_, dst_, align_, one_, kind_, sp_, dp_;
  int64_t fone_;
  int size_ = 0;
  std::vector<int32_t> pos_;
  std::vector<int64_t> taps_;
};

// utils.c get_local_pos: -513 (unset) means centred
int local_pos(int sub, int pos) {
  if (pos == -1 || pos <= -513) pos = (128 << sub) - 128;
  return (pos + 128) >> sub;
}

int ceil_rshift(int a, int b) { return -((-a) >> b); }

int64_t xinc(int src, int dst) { return (((int64_t)src << 16) + (dst >> 1)) / dst; }

void identity(SwsAxis* a, int n, int one, int shift) {
  a->size = a->eff = 1;
  a->n = n;
  a->pos.resize(n);
  a->coef.assign(n, (int16_t)one);
  for (int i = 0; i < n; i++) a->pos[i] = i >> shift;
}

int16_t round_to_int16(int64_t f) {  // utils.c roundToInt16
  const int r = (int)((f + (1 << 15)) >> 16);
  return (int16_t)(r < -0x7FFF ? -0x8000 : r > 0x7FFF ? 0x7FFF : r);
}

}  // namespace

SwsCsc sws_csc() {
  // ff_yuv2rgb_coeffs[SWS_CS_ITU601]; contrast = saturation = 1 << 16,
  // brightness 0; full range (yuvj: srcRange 1) scales the chroma terms
  int64_t crv = 104597, cbu = 132201, cgu = -25675, cgv = -53279;
  const int64_t cy = 1 << 16, oy = 0;
  crv = crv * 224 / 255;
  cbu = cbu * 224 / 255;
  cgu = cgu * 224 / 255;
  cgv = cgv * 224 / 255;
  SwsCsc c;
  c.y_coeff = round_to_int16(cy * (1 << 13));
  c.y_offset = round_to_int16(oy * (1 << 9));
  c.v2r = round_to_int16(crv * (1 << 13));
  c.v2g = round_to_int16(cgv * (1 << 13));
  c.u2g = round_to_int16(cgu * (1 << 13));
  c.u2b = round_to_int16(cbu * (1 << 13));
  c.crv = (int32_t)((crv * (1 << 16) + 0x8000) / cy);
  c.cbu = (int32_t)((cbu * (1 << 16) + 0x8000) / cy);
  c.cgu = (int32_t)((cgu * (1 << 16) + 0x8000) / cy);
  c.cgv = (int32_t)((cgv * (1 << 16) + 0x8000) / cy);
  return c;
}

int sws_plan(int srcW, int srcH, int hsub, int vsub, bool gray, int dstW, int dstH, int kind,
             SwsPlan* p) {
  *p = SwsPlan{};
  p->srcW = srcW;
  p->srcH = srcH;
  p->dstW = dstW;
  p->dstH = dstH;
  p->gray = gray;
  p->hsub = gray ? 0 : hsub;
  p->vsub = gray ? 0 : vsub;
  p->vmode.assign(dstH, kSwsX);
  const bool same = srcW == dstW && srcH == dstH;
  if (same && !gray && hsub == 1 && (vsub == 0 || (vsub == 1 && !(dstH & 1))) && !(dstW & 1)) {
    // yuv2rgb_c_24_rgb: nearest chroma (rows y >> vsub, pairs of columns)
    p->special = true;
    p->chrSrcW = p->chrDstW = ceil_rshift(srcW, hsub);
    p->chrSrcH = ceil_rshift(srcH, vsub);
    p->chrDstH = dstH;
    identity(&p->hl, dstW, 1 << 14, 0);
    identity(&p->vl, dstH, 1 << 12, 0);
    identity(&p->hc, p->chrDstW, 1 << 14, 0);
    identity(&p->vc, dstH, 1 << 12, vsub);
    p->vmode.assign(dstH, kSwsOne);
    return SPDL_HJ_OK;
  }
  p->full = (dstW & 1) || (p->hsub == 0 && p->vsub == 0);
  const int dst_hsub = p->full ? 0 : 1;
  p->chrSrcW = ceil_rshift(srcW, p->hsub);
  p->chrSrcH = ceil_rshift(srcH, p->vsub);
  p->chrDstW = ceil_rshift(dstW, dst_hsub);
  p->chrDstH = dstH;
  const int lp = local_pos(0, 0);
  if (!FilterBuilder((int)xinc(srcW, dstW), srcW, dstW, 4, 1 << 14, kind, lp, lp).build(&p->hl) ||
      !FilterBuilder((int)xinc(srcH, dstH), srcH, dstH, 2, 1 << 12, kind, lp, lp).build(&p->vl))
    return SPDL_HJ_ERR_BAD_GEOMETRY;
  if (!gray) {
    if (!FilterBuilder((int)xinc(p->chrSrcW, p->chrDstW), p->chrSrcW, p->chrDstW, 4, 1 << 14, kind,
                       local_pos(p->hsub, -513), local_pos(dst_hsub, -513))
             .build(&p->hc) ||
        !FilterBuilder((int)xinc(p->chrSrcH, p->chrDstH), p->chrSrcH, p->chrDstH, 2, 1 << 12, kind,
                       local_pos(p->vsub, -513), local_pos(0, -513))
             .build(&p->vc))
      return SPDL_HJ_ERR_BAD_GEOMETRY;
  }
  // packed_vscale's choice per output row
  const int lfs = p->vl.size, cfs = gray ? 1 : p->vc.size;
  for (int y = 0; y < dstH; y++) {
    const int16_t* lf = &p->vl.coef[(size_t)y * lfs];
    const int16_t* cf = gray ? nullptr : &p->vc.coef[(size_t)y * cfs];
    auto bilin = [](const int16_t* f) { return f[0] + f[1] == 4096 && (unsigned)f[1] <= 4096u; };
    int32_t m = kSwsX;
    if (gray) {
      if (lfs == 1) m = kSwsOne;
      else if (lfs == 2 && bilin(lf)) m = kSwsTwo | (lf[1] << 4);
    } else if (lfs == 1 && cfs == 1) {
      m = kSwsOne;
    } else if (lfs == 1 && cfs == 2 && bilin(cf)) {
      m = kSwsOne | (cf[1] << 17);
    } else if (lfs == 2 && cfs == 2 && bilin(lf) && bilin(cf)) {
      m = kSwsTwo | (lf[1] << 4) | (cf[1] << 17);
    }
    p->vmode[y] = m;
  }
  return SPDL_HJ_OK;
}

}  // namespace hj
