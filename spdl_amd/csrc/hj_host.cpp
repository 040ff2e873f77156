// hj_host.cpp -- host driver behind include/spdl_hipjpeg.h.
//
// Replaces src/libspdl/cuda/nvjpeg/decoding.cpp (decode_image_nvjpeg single
// :157-202 and batch :204-255) and src/libspdl/cuda/npp/detail/resize.cpp.
// Differences by design: the whole batch goes through one kernel
// sequence instead of a per-image nvjpegDecode + 3x nppiResize loop; the
// header probe replaces nvjpegGetImageInfo; bytes travel to HBM in one
// hipMemcpyAsync from pinned staging.
#include <hip/hip_runtime.h>

#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <tuple>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/spdl_hipjpeg.h"
#include "hj_common.h"
#include "hj_sws.h"

namespace hj {
hipError_t launch_parse(const uint8_t*, const ImageDesc*, ImageDesc*, ImageInfo*, HuffTable*,
                        const void*, void*, int64_t, const uint32_t*, uint32_t*, int, uint64_t*,
                        uint32_t*, uint32_t*, uint32_t*, uint32_t*, int, int, hipStream_t);
hipError_t launch_destuff(const uint8_t*, const ImageDesc*, ImageInfo*, DsChunk*, uint8_t*,
                          uint32_t*, const uint32_t*, int, int, int, hipStream_t);
hipError_t launch_entropy(const uint8_t*, const uint32_t*, const ImageDesc*, ImageInfo*,
                          const HuffTable*, uint32_t*, uint2*, uint32_t*, const uint32_t*, uint64_t*,
                          int, int, int, int, int, int64_t, hipStream_t);
hipError_t launch_idct(const uint32_t*, const uint2*, const ImageDesc*, const ImageInfo*, uint8_t*,
                       int, const uint32_t*, int, int, int, int, hipStream_t);
hipError_t launch_multiscan(const uint8_t*, uint8_t*, const ImageDesc*, ImageInfo*, uint32_t*, uint2*, int,
                            hipStream_t);
hipError_t launch_csc(const uint8_t*, const ImageDesc*, const ImageInfo*, void*,
                      const BatchParams&, int64_t, int, int32_t*, hipStream_t);
hipError_t launch_nv12(const uint8_t*, uint8_t*, int, int, int, int, int, hipStream_t);
hipError_t launch_sws(const uint8_t*, const ImageDesc*, const ImageInfo*, const int32_t*, void*,
                      const BatchParams&, const uint32_t*, int, int, int, int, int, int32_t*,
                      const uint32_t*, int, int16_t*, hipStream_t);
hipError_t launch_rgb_unscaled(const uint8_t*, const ImageDesc*, const ImageInfo*, void*,
                               const BatchParams&, int64_t, int, int32_t*, hipStream_t);
hipError_t launch_idct_rgb(const uint32_t*, const uint2*, const ImageDesc*, const ImageInfo*, void*,
                           const BatchParams&, int, int, int, int32_t*, hipStream_t);
hipError_t launch_cmyk(const ImageDesc*, const ImageInfo*, uint8_t*, int64_t, int, hipStream_t);
}  // namespace hj

using namespace hj;

namespace {

constexpr int kStages = 8;
const char* kStageNames[kStages] = {"h2d",  "parse",  "destuff", "entropy",
                                    "idct", "tables", "output",  "d2h_status"};

void set_err(char* err, size_t errlen, const char* fmt, ...) {
  if (!err || !errlen) return;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(err, errlen, fmt, ap);
  va_end(ap);
}

const char* status_str(int s) {
  switch (s) {
    case SPDL_HJ_OK: return "OK";
    case SPDL_HJ_ERR_NOT_JPEG: return "not a JPEG";
    case SPDL_HJ_ERR_UNSUPPORTED: return "unsupported JPEG (arithmetic, lossless, 12-bit or CMYK)";
    case SPDL_HJ_ERR_BAD_HEADER: return "corrupt JPEG header";
    case SPDL_HJ_ERR_BAD_HUFFMAN: return "corrupt entropy-coded data";
    case SPDL_HJ_ERR_TRUNCATED: return "truncated entropy-coded data";
    case SPDL_HJ_ERR_BAD_RESTART: return "restart marker mismatch";
    case SPDL_HJ_ERR_BAD_GEOMETRY: return "invalid resize geometry";
    case SPDL_HJ_ERR_INVALID_ARG: return "invalid argument";
    case SPDL_HJ_ERR_HIP: return "HIP runtime error";
    case SPDL_HJ_ERR_OOM: return "out of device memory";
    case SPDL_HJ_ERR_HANDOFF: return "entropy piece hand-off gave up";
    default: return "unknown error";
  }
}

inline int64_t round_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }

// A grow-only device buffer.  Given a stream, a growth is stream-ordered
// (hipFreeAsync / hipMallocAsync on it, after the work it already holds):
// hipFree synchronises the whole device, so a workspace that grew while a
// trainer's kernels ran on another stream used to wait for all of them (a
// decode beside a 0.46 s GEMM loop took 0.46 s; tests/test_gpu_pieces.py).
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t n, hipStream_t st = nullptr, bool async = false) {
    if (n <= cap) return hipSuccess;
    if (p) (void)(async ? hipFreeAsync(p, st) : hipFree(p));
    p = nullptr;
    cap = 0;
    size_t want = n + n / 4 + 4096;
    hipError_t e = async ? hipMallocAsync(&p, want, st) : hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// A grow-only pinned host buffer.  hipHostFree synchronises the whole
// device, so a buffer outgrown while the context runs is not freed then --
// that stalled a decode behind a trainer's kernels on another stream
// (tests/test_gpu_pieces.py: a 0.48 s GEMM loop) -- but kept until release();
// growth doubles, so the kept ones total less than the live buffer.
struct PinBuf {
  void* p = nullptr;
  void* dev = nullptr;  // the same pages as the device sees them (kernels read / write them)
  size_t cap = 0;
  std::vector<void*> old;  // outgrown buffers, freed by release()
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) old.push_back(p);
    p = dev = nullptr;
    const size_t want = std::max(2 * cap, n + n / 4 + 4096);
    cap = 0;
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e != hipSuccess) {
      p = nullptr;
      return e;
    }
    e = hipHostGetDevicePointer(&dev, p, 0);
    if (e != hipSuccess) {
      (void)hipHostFree(p);
      p = dev = nullptr;
      return e;
    }
    cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    for (void* q : old) (void)hipHostFree(q);
    old.clear();
    p = nullptr;
    dev = nullptr;
    cap = 0;
  }
};

// Persistent host workers for the pinned-staging copies.  A 256-image batch
// is ~28 MB; one core copies that at ~6-10 GB/s, slower than the GPU decodes
// it, so the copy into pinned memory is split over a few threads.
class CopyPool {
 public:
  explicit CopyPool(int n) {
    for (int i = 0; i < n; i++) th_.emplace_back([this, i] { loop(i + 1); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int workers() const { return (int)th_.size() + 1; }
  // fn(part, nparts) runs for part = 0..nparts-1 (part 0 on the caller).
  void run(const std::function<void(int, int)>& fn) {
    const int np = workers();
    {
      std::lock_guard<std::mutex> g(m_);
      fn_ = &fn;
      pending_ = np - 1;
      gen_++;
    }
    cv_.notify_all();
    fn(0, np);
    std::unique_lock<std::mutex> lk(m_);
    done_cv_.wait(lk, [this] { return pending_ == 0; });
    fn_ = nullptr;
  }

 private:
  void loop(int part) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int, int)>* fn;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        fn = fn_;
      }
      (*fn)(part, workers());
      std::lock_guard<std::mutex> g(m_);
      if (--pending_ == 0) done_cv_.notify_all();
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int, int)>* fn_ = nullptr;
  int pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// Copier threads per context: the host cores this process may use (affinity,
// capped by a cgroup v2 CPU quota) shared among the ranks of this node
// (LOCAL_WORLD_SIZE), at most 8 with the caller; SPDL_HJ_COPY_THREADS
// overrides.  8 ranks x 8 copiers would oversubscribe a 16-core share.
int copy_workers() {
  if (const char* e = getenv("SPDL_HJ_COPY_THREADS")) {
    const int v = atoi(e);
    return v < 1 ? 0 : (v > 16 ? 15 : v - 1);
  }
  int cores = (int)sysconf(_SC_NPROCESSORS_ONLN);
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) cores = CPU_COUNT(&set);
  if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    long long per = 0;
    if (fscanf(f, "%31s %lld", q, &per) == 2 && strcmp(q, "max") != 0 && per > 0) {
      const long long c = atoll(q) / per;
      if (c >= 1 && c < cores) cores = (int)c;
    }
    fclose(f);
  }
  int ranks = 1;
  if (const char* e = getenv("LOCAL_WORLD_SIZE")) ranks = atoi(e) > 0 ? atoi(e) : 1;
  const int share = cores / ranks;
  return share <= 1 ? 0 : (share - 1 > 7 ? 7 : share - 1);
}

// Copy n items of (dst_off, src, len) into `base`, zero-filling each item's
// tail [len, padded) -- split by bytes over the pool when the total is large.
struct CopyItem {
  int64_t dst_off;
  const uint8_t* src;
  int64_t len, padded;
};

void parallel_pack(CopyPool* pool, uint8_t* base, const std::vector<CopyItem>& items) {
  int64_t total = 0;
  for (const CopyItem& it : items) total += it.padded;
  auto body = [&](int part, int np) {
    // byte range [lo, hi) of the concatenated padded items
    const int64_t lo = total * part / np, hi = total * (part + 1) / np;
    int64_t acc = 0;
    for (const CopyItem& it : items) {
      const int64_t a = acc, b = acc + it.padded;
      acc = b;
      if (b <= lo) continue;
      if (a >= hi) break;
      const int64_t s = lo > a ? lo - a : 0, e = (hi < b ? hi : b) - a;
      const int64_t cs = s, ce = e < it.len ? e : it.len;
      if (ce > cs) memcpy(base + it.dst_off + cs, it.src + cs, (size_t)(ce - cs));
      const int64_t zs = s > it.len ? s : it.len;
      if (e > zs) memset(base + it.dst_off + zs, 0, (size_t)(e - zs));
    }
  };
  if (!pool || pool->workers() < 2 || total < (4 << 20)) body(0, 1);
  else pool->run(body);
}

// Components of the first scan (SOS Ns) after `pos`; 255 when no SOS header
// follows (the device parse then reports the file).
int first_scan_components(const uint8_t* d, size_t size, size_t pos) {
  for (;;) {
    while (pos < size && d[pos] != 0xFF) pos++;
    while (pos < size && d[pos] == 0xFF) pos++;
    if (pos >= size) return 255;
    const int m = d[pos++];
    if (m == 0x01 || (m >= 0xD0 && m <= 0xD8)) continue;
    if (m == 0xD9 || pos + 3 > size) return 255;
    if (m == 0xDA) return d[pos + 2];
    pos += (size_t)((d[pos] << 8) | d[pos + 1]);
  }
}

// ---- host SOF probe (replaces nvjpegGetImageInfo) --------------------------
// The SOF fields and the frame's colour model (frame_color: the APP14 Adobe
// flag seen before the SOF, the component ids).
int probe(const uint8_t* d, size_t size, spdl_hj_image_info* info) {
  memset(info, 0, sizeof(*info));
  if (!d || size < 4 || d[0] != 0xFF || d[1] != 0xD8) return SPDL_HJ_ERR_NOT_JPEG;
  size_t pos = 2;
  int adobe = -1;
  for (;;) {
    while (pos < size && d[pos] != 0xFF) pos++;
    while (pos < size && d[pos] == 0xFF) pos++;
    if (pos >= size) return SPDL_HJ_ERR_BAD_HEADER;
    int m = d[pos++];
    if (m == 0xD8 || m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;
    if (m == 0xD9 || m == 0xDA) return SPDL_HJ_ERR_BAD_HEADER;  // no SOF before the scan
    if (pos + 2 > size) return SPDL_HJ_ERR_BAD_HEADER;
    int len = (d[pos] << 8) | d[pos + 1];
    if (len < 2 || pos + (size_t)len > size) return SPDL_HJ_ERR_BAD_HEADER;
    const uint8_t* s = d + pos + 2;
    pos += (size_t)len;
    if (m == 0xEE) {
      if (len >= 14 && memcmp(s, "Adobe", 5) == 0) adobe = s[11];
      continue;
    }
    if (m == 0xC0 || m == 0xC1 || m == 0xC2) {  // sequential or progressive Huffman
      if (len < 8) return SPDL_HJ_ERR_BAD_HEADER;
      if (s[0] != 8) return SPDL_HJ_ERR_UNSUPPORTED;
      info->height = (s[1] << 8) | s[2];
      info->width = (s[3] << 8) | s[4];
      info->ncomp = s[5];
      if (info->height == 0) return SPDL_HJ_ERR_UNSUPPORTED;
      if (info->width == 0) return SPDL_HJ_ERR_BAD_HEADER;
      if (info->ncomp != 1 && info->ncomp != 3 && info->ncomp != 4) return SPDL_HJ_ERR_UNSUPPORTED;
      if (len < 8 + 3 * info->ncomp) return SPDL_HJ_ERR_BAD_HEADER;
      int ids[kMaxComp] = {};
      for (int c = 0; c < info->ncomp; c++) {
        ids[c] = s[6 + 3 * c];
        info->h_samp[c] = s[7 + 3 * c] >> 4;
        info->v_samp[c] = s[7 + 3 * c] & 15;
        if (info->h_samp[c] < 1 || info->h_samp[c] > 4 || info->v_samp[c] < 1 ||
            info->v_samp[c] > 4)
          return SPDL_HJ_ERR_BAD_HEADER;
      }
      if (!frame_color(info->ncomp, info->h_samp, info->v_samp, ids, adobe, &info->color))
        return SPDL_HJ_ERR_UNSUPPORTED;
      // the scan structure: progressive, or a first scan with fewer
      // components than the frame (the multi-scan path decodes both)
      info->multiscan = m == 0xC2 || first_scan_components(d, size, pos) < info->ncomp;
      return SPDL_HJ_OK;
    }
    if (m == 0xC3 || (m >= 0xC5 && m <= 0xC7) || (m >= 0xC9 && m <= 0xCB) ||
        (m >= 0xCD && m <= 0xCF))
      return SPDL_HJ_ERR_UNSUPPORTED;  // lossless, hierarchical, arithmetic
  }
}

// ---- geometry (FFmpeg scale/pad/crop semantics; see oracle jo_geometry) ----
int64_t rescale_rnd(int64_t a, int64_t b, int64_t c) { return (a * b + c / 2) / c; }

struct Geom {
  int sw, sh, dx, dy, ow, oh;
};

int geometry(int w, int h, const spdl_hj_output* o, Geom* g) {
  if (w <= 0 || h <= 0) return SPDL_HJ_ERR_BAD_GEOMETRY;
  if (!o->resize) {
    *g = {w, h, 0, 0, w, h};
    return SPDL_HJ_OK;
  }
  int64_t fw = o->fit_w > 0 ? o->fit_w : w, fh = o->fit_h > 0 ? o->fit_h : h;
  int64_t sw = fw, sh = fh;
  if (o->aspect != SPDL_HJ_ASPECT_NONE) {
    int64_t tw = rescale_rnd(fh, w, h), th = rescale_rnd(fw, h, w);
    if (o->aspect == SPDL_HJ_ASPECT_DECREASE) {
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
  if (o->pad_w > 0 && o->pad_h > 0) {
    cw = o->pad_w;
    ch = o->pad_h;
    if (cw < sw || ch < sh) return SPDL_HJ_ERR_BAD_GEOMETRY;
    px = (cw - sw) / 2;
    py = (ch - sh) / 2;
  }
  int64_t ow = cw, oh = ch, cx = 0, cy = 0;
  if (o->crop_w > 0 && o->crop_h > 0) {
    ow = o->crop_w;
    oh = o->crop_h;
    if (ow > cw || oh > ch) return SPDL_HJ_ERR_BAD_GEOMETRY;
    cx = (cw - ow) / 2;
    cy = (ch - oh) / 2;
  }
  if (sw > 65535 || sh > 65535 || ow > 65535 || oh > 65535) return SPDL_HJ_ERR_BAD_GEOMETRY;
  *g = {(int)sw, (int)sh, (int)(px - cx), (int)(py - cy), (int)ow, (int)oh};
  return SPDL_HJ_OK;
}

// ---- swscale plans (hj_sws.h), packed for the device ----------------------
// One per distinct (source size, sampling, output placement, filter); cached
// per context so a stream of same-size images plans once.
enum { kPlanYuv = 0, kPlanGray = 1, kPlanGbr = 2 };  // source planes of a plan
struct PlanKey {
  int w, h, hsub, vsub, mode, filter, sw, sh, dx, dy, ow, oh;
  bool operator<(const PlanKey& o) const {
    return std::tie(w, h, hsub, vsub, mode, filter, sw, sh, dx, dy, ow, oh) <
           std::tie(o.w, o.h, o.hsub, o.vsub, o.mode, o.filter, o.sw, o.sh, o.dx, o.dy, o.ow, o.oh);
  }
};

struct PackedPlan {
  SwsDesc d{};                  // offsets relative to the blob
  std::vector<int32_t> blob;    // tables, 16-byte aligned sections
  int bands = 0, chunks = 0, lds = 0;
  bool special = false;         // swscale's unscaled yuv2rgb_c_24_rgb converter
};

class PlanCache {
 public:
  // the horizontal pass of large downscales in hscale_kernel (SwsDesc::pre):
  // -1 when the vertical ratio is >= kPreRatio or the luma filter is longer
  // than the kernel's register buckets (64 taps), 0 never, 1 always
  // (spdl_hj_set_param "sws_prepass"; outputs are identical)
  static constexpr int kPreRatio = 4;
  void set_pre_mode(int m) {
    if (m != pre_mode_) map_.clear();
    pre_mode_ = m;
  }
  int pre_mode() const { return pre_mode_; }
  // widest column chunk a tile may take (16-256; the tiler then picks the
  // tallest band that fits the LDS budget)
  void set_max_cols(int c) {
    if (c != max_cols_) map_.clear();
    max_cols_ = c;
  }
  int max_cols() const { return max_cols_; }
  std::shared_ptr<const PackedPlan> get(const PlanKey& k, int* rc) {
    auto it = map_.find(k);
    if (it != map_.end()) return it->second;
    auto p = build(k, rc, pre_mode_, max_cols_);
    if (!p) return nullptr;
    if (map_.size() >= 512) map_.clear();  // bounded: a stream of odd sizes replans
    map_.emplace(k, p);
    return p;
  }

 private:
  static void put(std::vector<int32_t>& blob, int32_t* off, const void* data, size_t bytes) {
    *off = (int32_t)blob.size();
    const size_t words = (bytes + 3) / 4;
    blob.resize(blob.size() + ((words + 3) & ~(size_t)3), 0);
    if (bytes) memcpy(blob.data() + *off, data, bytes);
  }

  static std::shared_ptr<const PackedPlan> build(const PlanKey& k, int* rc, int pre_mode,
                                                 int max_cols) {
    SwsPlan pl;
    // gbr: the luma plan (gray) applied to each of the three RGB planes
    *rc = sws_plan(k.w, k.h, k.hsub, k.vsub, k.mode != kPlanYuv, k.sw, k.sh, k.filter, &pl);
    if (*rc) return nullptr;
    auto pp = std::make_shared<PackedPlan>();
    pp->special = pl.special && k.dx == 0 && k.dy == 0 && k.ow == k.sw && k.oh == k.sh;
    SwsDesc& d = pp->d;
    d.sw = k.sw;
    d.sh = k.sh;
    d.chr_w = pl.chrDstW;
    d.full = pl.full;
    d.gray = pl.gray;
    d.gbr = k.mode == kPlanGbr;
    const SwsAxis* ax[4] = {&pl.hl, &pl.hc, &pl.vl, &pl.vc};
    int32_t* taps[4] = {&d.hl_taps, &d.hc_taps, &d.vl_taps, &d.vc_taps};
    int32_t* sizes[4] = {&d.hl_size, &d.hc_size, &d.vl_size, &d.vc_size};
    for (int i = 0; i < 4; i++) {
      // rows cut to the taps that are ever non-zero, padded to a multiple
      // of 4 (the kernel reads taps 4 at a time)
      const SwsAxis& a = *ax[i];
      const int eff = a.eff;
      // horizontal rows: padded to the kernel's register bucket of taps
      // (hpass: 4, 8, 12, 16, 24, 32, 48, 64; longer rows use a plain loop)
      int q = (eff + 3) / 4;
      if (i < 2) q = q <= 4 ? q : q <= 6 ? 6 : q <= 8 ? 8 : q <= 12 ? 12 : q <= 16 ? 16 : q;
      const int stride = 4 * q;
      *taps[i] = eff;
      *sizes[i] = stride;
      std::vector<int16_t> rows((size_t)a.n * stride, 0);
      for (int r = 0; r < a.n; r++)
        for (int t = 0; t < eff; t++) rows[(size_t)r * stride + t] = a.coef[(size_t)r * a.size + t];
      put(pp->blob, &d.off[2 * i], a.pos.data(), a.pos.size() * 4);
      put(pp->blob, &d.off[2 * i + 1], rows.data(), rows.size() * 2);
    }
    put(pp->blob, &d.off[kVmode], pl.vmode.data(), pl.vmode.size() * 4);
    // source rows the vertical filters reach (first tap + taps, max over rows)
    auto reach = [](const SwsAxis& a) {
      int r = 0;
      for (int y = 0; y < a.n; y++) r = std::max(r, a.pos[y] + a.eff);
      return r;
    };
    d.pre = pre_mode > 0 ||
            (pre_mode < 0 && !pp->special && (k.h >= kPreRatio * k.sh || pl.hl.eff > 64));
    d.pre_rl = d.pre ? reach(pl.vl) : 0;
    d.pre_rc = d.pre && !pl.gray ? reach(pl.vc) : 0;
    // tiling: the tallest band (and widest column chunk) whose horizontal
    // pass rows (+ 4 slack rows) and u8 output tile fit the LDS budget;
    // bands are in output rows
    for (int cols = std::min(max_cols, kSwsMaxCols); cols >= 16 && !pp->bands; cols /= 2) {
      const int chunk = k.ow < cols ? k.ow : cols;
      static const int kRb[] = {32, 24, 16, 12, 8, 6, 4, 3, 2, 1};
      for (int rb : kRb) {
        int64_t lds = 0;
        for (int yo0 = 0; yo0 < k.oh; yo0 += rb) {
          const int ys0 = std::max(yo0 - k.dy, 0), ys1 = std::min(yo0 + rb - k.dy, k.sh);
          if (ys0 >= ys1) continue;
          const int64_t lrows = pl.vl.pos[ys1 - 1] + pl.vl.eff - pl.vl.pos[ys0];
          const int64_t crows = pl.gray ? 0 : pl.vc.pos[ys1 - 1] + pl.vc.eff - pl.vc.pos[ys0];
          for (int xo0 = 0; xo0 < k.ow; xo0 += chunk) {
            const int xs0 = std::max(xo0 - k.dx, 0), xs1 = std::min(xo0 + chunk - k.dx, k.sw);
            if (xs0 >= xs1) continue;
            const int64_t ncl = xs1 - xs0;
            const int64_t ncc = pl.gray ? 0 : pl.full ? ncl : ((xs1 - 1) >> 1) - (xs0 >> 1) + 1;
            const int64_t h = 2 * ((d.gbr ? 3 : 1) * ncl * sws_col_stride((int)lrows) +
                                   (pl.gray ? 0 : 2 * ncc * sws_col_stride((int)crows)));
            lds = std::max(lds, (h + 15) & ~(int64_t)15);
          }
        }
        // + the u8 output tile and the band's staged vertical tables
        const int64_t tile = (((int64_t)rb * chunk * 3 + 15) & ~(int64_t)15) +
                             (int64_t)rb * (16 + 2 * (d.vl_size + d.vc_size));
        // (the launch's LDS is the batch's largest plan's: a plan over the
        // budget slows every image's tiles; only a one-row band of a plan
        // without the hscale pre-pass may exceed it)
        if (lds + tile <= kSwsLdsBudget || (!d.pre && rb == 1 && lds + tile <= 64 * 1024)) {
          d.rb = rb;
          d.col_chunk = chunk;
          pp->lds = (int)(lds + tile);
          pp->bands = (k.oh + rb - 1) / rb;
          pp->chunks = (k.ow + chunk - 1) / chunk;
          break;
        }
      }
    }
    if (!pp->bands) {
      *rc = SPDL_HJ_ERR_BAD_GEOMETRY;
      return nullptr;
    }
    return pp;
  }

  std::map<PlanKey, std::shared_ptr<const PackedPlan>> map_;
  int pre_mode_ = -1;
  int max_cols_ = kSwsMaxCols;
};

// chroma subsampling shifts of the yuvj4xxp frame FFmpeg's mjpeg decoder
// makes of this sampling (444 / 422 / 420 / 440 / 411 ...); others are not
// a swscale input format here
int chroma_shifts(const spdl_hj_image_info& p, int* hs, int* vs) {
  *hs = *vs = 0;
  if (p.ncomp != 3) return SPDL_HJ_OK;  // gray, or 4 components all 1x1 (probe)
  const int hmax = std::max(p.h_samp[0], std::max(p.h_samp[1], p.h_samp[2]));
  const int vmax = std::max(p.v_samp[0], std::max(p.v_samp[1], p.v_samp[2]));
  if (p.h_samp[0] != hmax || p.v_samp[0] != vmax || p.h_samp[1] != p.h_samp[2] ||
      p.v_samp[1] != p.v_samp[2] || hmax % p.h_samp[1] || vmax % p.v_samp[1])
    return SPDL_HJ_ERR_UNSUPPORTED;
  const int rh = hmax / p.h_samp[1], rv = vmax / p.v_samp[1];
  if ((rh & (rh - 1)) || (rv & (rv - 1))) return SPDL_HJ_ERR_UNSUPPORTED;
  while ((1 << *hs) < rh) (*hs)++;
  while ((1 << *vs) < rv) (*vs)++;
  return SPDL_HJ_OK;
}

struct Layout {
  std::vector<ImageDesc> desc;
  std::vector<int32_t> tables;  // the batch's swscale table pool
  int64_t total_blocks = 0, total_planes = 0, total_segs = 0, total_recs = 0;
  int64_t out_elems_per_image = 0;
  int max_blocks = 0;
  int64_t max_px = 0;
  int64_t total_ds = 0;
  int max_chunks = 0;
  int ow = 0, oh = 0;
  int sws_bands = 0, sws_chunks = 0, sws_lds = 0;
  bool all_special = true;  // every image takes swscale's unscaled converter
  bool fuse_ok = true;      // ... with standard 4:2:0 / 4:2:2 MCUs (idct_rgb_kernel)
  int64_t cmyk_px = 0;      // 4-component images needing cmyk_kernel's K transform: max pixels
  int fused_tiles = 0;      // idct_rgb_kernel workgroups per image (max)
  // entropy work items (image | piece << 24), the images with the most
  // pieces first, and the granules of their hand-off records (hj_common.h)
  std::vector<uint32_t> work;
  int64_t chain_granules = 0;
  // flat destuff / IDCT grids: workgroups over the whole batch
  int64_t ds_wgs = 0, idct_wgs = 0;
  // hscale_kernel (large downscales): workgroups and int16 rows
  int64_t hs_wgs = 0, total_hbuf = 0;
  int64_t sws_wgs = 0;  // sws_kernel tiles over the batch (per-image plans)
  // a progressive (SOF2) image is in the batch: multiscan_kernel runs on a
  // side stream beside destuff + entropy (only the host-bytes entry points
  // see the headers; elsewhere it runs after entropy on the lane's stream)
  bool ms_side = false;
  // the entry point knows every image's scan structure (host probes, or the
  // caller's ABI-5 image_info): a batch without multi-scan images may skip
  // the multi-scan launch
  bool ms_known = false;
  // images decoded by several entropy workgroups (hand-offs): their probes,
  // for a one-workgroup re-decode should a hand-off give up
  std::vector<std::pair<int, spdl_hj_image_info>> multi;
};

int build_layout(const int64_t* offsets, const int64_t* sizes, const spdl_hj_image_info* infos,
                 int n, const spdl_hj_output* out, int sub_bits, int64_t piece_bytes, Layout& L,
                 int32_t* status, char* err, size_t errlen, PlanCache* plans) {
  L.desc.assign(n, ImageDesc{});
  // plan -> offset in L.tables.  `alive` holds every placed plan until the
  // layout is built: the cache may evict (and free) a plan mid-batch, and a
  // new plan at a recycled address must not match a stale `placed` entry
  std::map<const PackedPlan*, int64_t> placed;
  std::vector<std::shared_ptr<const PackedPlan>> alive;
  auto fail = [&](int i, int rc, const char* what) {
    if (status) status[i] = rc;
    set_err(err, errlen, "Failed to decode an image. (image %d: %s)", i, what ? what : status_str(rc));
    return rc;
  };
  for (int i = 0; i < n; i++) {
    ImageDesc& d = L.desc[i];
    const spdl_hj_image_info& p = infos[i];
    d.in_off = offsets[i];
    d.in_size = sizes[i];
    d.width = p.width;
    d.height = p.height;
    d.ncomp = p.ncomp;
    d.color = p.color;
    if (p.ncomp == 4) {
      // libjpeg's JFIF conversion has no CMYK -> RGB; the K transform
      // (FFmpeg's, cmyk_kernel) runs unless the planes are YCbCr + K
      if (out->csc == SPDL_HJ_CSC_JFIF) return fail(i, SPDL_HJ_ERR_UNSUPPORTED, "CMYK with csc=jfif");
      if (p.color != kColorYcbcrk) L.cmyk_px = std::max(L.cmyk_px, (int64_t)p.width * p.height);
    }
    int hmax = 1, vmax = 1;
    for (int c = 0; c < p.ncomp; c++) {
      d.h_samp[c] = p.h_samp[c];
      d.v_samp[c] = p.v_samp[c];
      hmax = p.h_samp[c] > hmax ? p.h_samp[c] : hmax;
      vmax = p.v_samp[c] > vmax ? p.v_samp[c] : vmax;
    }
    int bw[kMaxComp] = {}, bh[kMaxComp] = {};
    int64_t nblocks;
    if (p.ncomp == 1) {
      bw[0] = (p.width + 7) / 8;
      bh[0] = (p.height + 7) / 8;
      nblocks = (int64_t)bw[0] * bh[0];
    } else {
      int mcux = (p.width + 8 * hmax - 1) / (8 * hmax), mcuy = (p.height + 8 * vmax - 1) / (8 * vmax);
      int bpm = 0;
      for (int c = 0; c < p.ncomp; c++) {
        if (hmax % p.h_samp[c] || vmax % p.v_samp[c]) return fail(i, SPDL_HJ_ERR_UNSUPPORTED, nullptr);
        bw[c] = mcux * p.h_samp[c];
        bh[c] = mcuy * p.v_samp[c];
        bpm += p.h_samp[c] * p.v_samp[c];
      }
      if (bpm > kMaxBpm) return fail(i, SPDL_HJ_ERR_UNSUPPORTED, nullptr);
      nblocks = (int64_t)mcux * mcuy * bpm;
    }
    // the entropy kernel's 32-bit byte offsets into an image's coefficient
    // lists (4 bytes x 64 entries per block) must not wrap
    if (nblocks >= (1 << 24)) return fail(i, SPDL_HJ_ERR_UNSUPPORTED, "image too large");
    d.nblocks = (int)nblocks;
    d.coef_off = L.total_blocks;
    L.total_blocks += nblocks;
    if (d.nblocks > L.max_blocks) L.max_blocks = d.nblocks;
    for (int c = 0; c < p.ncomp; c++) {
      d.plane_stride[c] = bw[c] * 8;
      d.plane_off[c] = L.total_planes;
      L.total_planes += round_up((int64_t)bw[c] * 8 * bh[c] * 8, 256);
    }
    d.seg_cap = (int32_t)(sizes[i] / 2 + 2);
    d.seg_off = L.total_segs;
    L.total_segs += d.seg_cap;
    d.ds_cap = (int32_t)(sizes[i] / kDsChunk + 2);
    d.ds_off = L.total_ds;
    L.total_ds += d.ds_cap;
    d.ds_wg0 = (int32_t)L.ds_wgs;
    L.ds_wgs += d.ds_cap;
    d.idct_wg0 = (int32_t)L.idct_wgs;
    L.idct_wgs += (nblocks + kIdctThreads - 1) / kIdctThreads;
    if (d.ds_cap > L.max_chunks) L.max_chunks = d.ds_cap;
    // size-adaptive entropy decode: a file larger than piece_bytes is
    // decoded by ceil(size / piece_bytes) workgroups (progressive and
    // multi-scan images take multiscan_kernel: one)
    int pieces = 1;
    if (piece_bytes > 0 && !p.multiscan && sizes[i] > piece_bytes)
      pieces = (int)std::min<int64_t>(kMaxPieces, (sizes[i] + piece_bytes - 1) / piece_bytes);
    d.pieces = pieces;
    d.chain_off = pieces > 1 ? (int32_t)L.chain_granules : 0;
    if (pieces > 1) {
      L.chain_granules += (int64_t)pieces * kChainGranules;
      L.multi.emplace_back(i, p);
    }
    // entropy slot state (u32 units): kMaxSlots uint4 + slack per piece
    d.rec_cap = (int64_t)kMaxSlots * 8 * pieces;
    d.rec_off = L.total_recs;
    L.total_recs += d.rec_cap;
    Geom g;
    int rc = geometry(p.width, p.height, out, &g);
    if (rc) return fail(i, rc, nullptr);
    d.dx = g.dx;
    d.dy = g.dy;
    d.ow = g.ow;
    d.oh = g.oh;
    if (i == 0) {
      L.ow = g.ow;
      L.oh = g.oh;
    } else if (g.ow != L.ow || g.oh != L.oh) {
      set_err(err, errlen,
              "all images of a batch must produce the same output size "
              "(image 0: %dx%d, image %d: %dx%d); pass a resize target",
              L.ow, L.oh, i, g.ow, g.oh);
      return SPDL_HJ_ERR_INVALID_ARG;
    }
    int64_t px = (int64_t)g.ow * g.oh;
    if (px > L.max_px) L.max_px = px;
    if (!plans || out->csc == SPDL_HJ_CSC_JFIF) continue;
    int hs, vs;
    if ((rc = chroma_shifts(p, &hs, &vs))) return fail(i, rc, nullptr);
    // RGB planes (gbrp; CMYK after the K transform, gbrap) through the luma
    // filters; YCCK after the transform and YCbCr + K are YCbCr 4:4:4
    const int mode = p.ncomp == 1                                        ? kPlanGray
                     : p.color == kColorRgb || p.color == kColorCmyk ? kPlanGbr
                                                                      : kPlanYuv;
    const PlanKey key{p.width, p.height, hs, vs, mode, out->resize ? out->filter : 0,
                      g.sw, g.sh, g.dx, g.dy, g.ow, g.oh};
    auto plan = plans->get(key, &rc);
    if (!plan) return fail(i, rc, rc == SPDL_HJ_ERR_BAD_GEOMETRY ? "scale filter too long" : nullptr);
    auto it = placed.find(plan.get());
    if (it == placed.end()) {
      it = placed.emplace(plan.get(), (int64_t)L.tables.size()).first;
      alive.push_back(plan);
      L.tables.insert(L.tables.end(), plan->blob.begin(), plan->blob.end());
    }
    d.wt_off = it->second;
    d.sws = plan->d;
    if (plan->d.pre) {  // hscale_kernel rows: luma, then the two chroma planes
      const SwsDesc& sd = plan->d;
      const int wc = sd.gbr ? sd.sw : sd.chr_w, rc = sd.gbr ? sd.pre_rl : sd.pre_rc;
      const int tl = (sd.pre_rl + kHsRows - 1) / kHsRows;
      const bool chroma = sd.gbr || !sd.gray;  // (gbr plans are gray plans on three planes)
      const int tc = chroma ? (rc + kHsRows - 1) / kHsRows : 0;
      d.hs_wg0 = (int32_t)L.hs_wgs;
      d.hs_wgs = tl + 2 * tc;
      L.hs_wgs += d.hs_wgs;
      d.hbuf_off = L.total_hbuf;
      L.total_hbuf += (int64_t)sd.pre_rl * sd.sw + (chroma ? 2 * (int64_t)rc * wc : 0);
    }
    L.all_special = L.all_special && plan->special;
    // idct_rgb_kernel's MCU shapes: Y 2x2 or 2x1, U and V 1x1
    if (p.ncomp == 3 && p.h_samp[0] == 2 && (p.v_samp[0] == 1 || p.v_samp[0] == 2) &&
        p.h_samp[1] == 1 && p.v_samp[1] == 1 && p.h_samp[2] == 1 && p.v_samp[2] == 1) {
      const int bpm = 2 * p.v_samp[0] + 2, tw = kFusedThreads / bpm;
      const int mcux = (p.width + 15) / 16, mcuy = (p.height + 8 * p.v_samp[0] - 1) / (8 * p.v_samp[0]);
      L.fused_tiles = std::max(L.fused_tiles, (mcux + tw - 1) / tw * mcuy);
    } else {
      L.fuse_ok = false;
    }
    L.sws_bands = std::max(L.sws_bands, plan->bands);
    L.sws_chunks = std::max(L.sws_chunks, plan->chunks);
    d.sws_wg0 = (int32_t)L.sws_wgs;  // flat sws grid: this image's tiles only
    d.sws_bands = plan->bands;
    d.sws_chunks = plan->chunks;
    L.sws_wgs += (int64_t)plan->bands * plan->chunks;
    L.sws_lds = std::max(L.sws_lds, plan->lds);
  }
  L.out_elems_per_image = (int64_t)L.ow * L.oh * 3;
  for (int i = 0; i < n; i++) L.desc[i].out_off = (int64_t)i * L.out_elems_per_image;
  // entropy work list: the images with the most pieces first (their pieces
  // start early and in ticket order), each image's pieces in order
  std::vector<int> order(n);
  for (int i = 0; i < n; i++) order[i] = i;
  std::stable_sort(order.begin(), order.end(),
                   [&](int a, int b) { return L.desc[a].pieces > L.desc[b].pieces; });
  L.work.clear();
  for (int i : order)
    for (int q = 0; q < L.desc[i].pieces; q++) L.work.push_back((uint32_t)i | ((uint32_t)q << 24));
  return SPDL_HJ_OK;
}

}  // namespace

// One in-flight batch: pinned staging + device copy of the JPEG bytes, the
// descriptor/status staging, and the events that say when each may be reused.
// kSlots of them form the ring that lets batch k+1 be packed on the host and
// copied (on the context's copy stream) while batch k's kernels run.
constexpr int kSlots = 10;

struct Slot {
  PinBuf pin_in, pin_desc, pin_status, pin_tables;
  DevBuf bytes;
  hipEvent_t h2d_done = nullptr;  // bytes are in HBM
  hipEvent_t done = nullptr;      // the batch's last kernel / status copy finished
  int64_t ticket = 0;             // ticket of the batch occupying the slot (0 = none)
  bool pending = false;           // submitted, not yet waited
  bool staged = false;            // acquired by spdl_hj_staging_acquire, not submitted
  bool profiled = false;          // ev[] were recorded for this batch
  uint32_t profiled_stages = 0;   // ... for these stages
  hipEvent_t submitted = nullptr; // lanes > 1: the caller's stream reached the submit
  int n = 0;
  hipEvent_t ev[kStages + 1] = {};  // stage boundaries (profiling only)
  // A batch with multi-piece images: what re-decoding one of them in one
  // workgroup needs, should a piece hand-off give up (kErrHandoff)
  struct Retry {
    int64_t ticket = 0;              // the batch's (its lane's workspace)
    const uint8_t* bytes = nullptr;  // the batch's bytes in HBM
    size_t len = 0;
    spdl_hj_output out{};
    uint8_t* out_dev = nullptr;
    size_t img_bytes = 0;  // output bytes per image
    std::vector<int> idx;
    std::vector<int64_t> off, size;
    std::vector<spdl_hj_image_info> info;
  } retry;
};

// Device workspace of one pipeline "lane".  With lanes > 1 successive
// batches alternate between workspaces and run on the lanes' own streams, so
// batch k+1's kernels can occupy the CUs that batch k's latency-bound
// entropy kernel leaves idle (its sync rounds park most waves at barriers).
constexpr int kMaxLanes = 8;

struct Workspace {
  DevBuf clean, segs, desc, info, luts, ents, bdesc, planes, wts, recs, dschunks;
  DevBuf chain;  // entropy ticket counter + piece hand-off records (hj_common.h)
  DevBuf maps;   // flat-grid dispatch maps: destuff chunks, IDCT tiles, hscale rows -> image
  DevBuf hbuf;   // hscale_kernel's horizontal-pass rows (large downscales)
  hipEvent_t done = nullptr;      // the workspace is free after this
  hipStream_t stream = nullptr;   // lanes > 1 only
  // multiscan_kernel beside the baseline stages (batches with a progressive
  // image, host-bytes entry points): created on first use
  hipStream_t side = nullptr;
  hipEvent_t ev_parsed = nullptr, ev_ms = nullptr;
  hipStream_t last_st = nullptr;  // the stream the workspace's last batch ran on
  bool used = false;
};

struct spdl_hj_ctx {
  int device = 0;
  Workspace ws[kMaxLanes];
  int lanes = 1;
  // the ring, and a spare slot outside it for the one-workgroup re-decode of
  // an image whose piece hand-off gave up (it must not take a ring slot a
  // caller's un-waited ticket may still hold)
  Slot slots[kSlots + 1];
  int64_t next_ticket = 1;
  int64_t last_ticket = 0;
  int lanes_ready = 0;                // workspaces [0, lanes_ready) have their event / stream
  hipStream_t copy = nullptr;         // H2D stream of the staging ring
  CopyPool* pool = nullptr;           // created on the first large host copy
  // hardware queues HIP gives this process (GPU_MAX_HW_QUEUES when HIP
  // initialised; 4 is HIP's default): each lane's stream wants one of its own
  int hw_queues = 4;
  // stream priority of the lanes' streams: 1 low (default), 0 normal, -1
  // high.  HIP keeps a pool of up to GPU_MAX_HW_QUEUES hardware queues per
  // priority, so low-priority lanes get queues of their own beside the
  // normal-priority pool that the null stream, torch's streams and the copy
  // stream share (measured with 4 queues, 4 lanes: 408k img/s at normal
  // priority -- the lanes landed on two queues -- 508k at low, as with 16).
  // Multiscan side streams are high priority (a third pool): they carry the
  // mixed batch's critical path.
  int lane_priority = 1;
  // output kernels: 0 = by batch (fused IDCT + converter at full resolution
  // when possible), 1 = the generic swscale kernel, 2 = separate IDCT +
  // unscaled converter -- byte-identical outputs (tests compare them)
  int output_path = 0;
  bool profiling = false;
  // stages whose HIP events are recorded while profiling (bit i: stage i of
  // kStageNames; a bench brackets only its dominant kernel in the timed steps)
  uint32_t profile_stages = (1u << kStages) - 1u;
  float timings[kStages] = {};
  int ntimings = 0;
  int sub_bits = 384;
  int debug_mask = 0;  // timing ablations, settable only in HJ_ABLATIONS builds
  // the first kernel pulls descriptors + tables from pinned memory and the
  // last writes statuses back (1), or DMA copies do it (0; kept for A/B)
  int host_staging = 1;
  // Huffman workgroup size; 0 = by schedule: 512 with one lane (shortest
  // kernel), 256 with two or more (the smaller workgroups leave the other
  // lane's kernels more room: +3 % in the 2-lane bench, r02 A/B)
  int entropy_threads = 0;
  // entropy round 0: slots decoded before a run's first slot; -1 = by
  // workgroup size: 12 with 512+ threads, 6 with 256 (each run then spans
  // twice the slots; 4-lane A/B: 459-461k vs 450-454k img/s, r02_v5)
  int warm_slots = -1;
  // entropy piece size: a file larger than this is decoded by several
  // workgroups (hj_common.h kMaxPieces); 0 = one workgroup per image
  int64_t piece_bytes = 128 * 1024;
  // entropy runs hold at least this many slots (0: one run per thread)
  int min_run_slots = 0;
  // entropy sync rounds after which unresolved chains are re-decoded by
  // whole waves (chain rounds; 0 = never; -1 = by workgroup size: 1 with
  // 512+ threads, 2 with 256).  r06: the mixed set's slowest image (q94,
  // optimised tables, 11 sync rounds) 1.02 -> 0.63 ms alone, one-lane mixed
  // entropy 0.90 -> 0.69 ms; at one lane 1 also takes the uniform batch's
  // entropy 0.450 -> 0.434 ms (318 k -> 325 k img/s); at four lanes 2 and 1
  // measure the same (profiles/r06/ab/warm_chain.txt)
  int chain_after = -1;
  // s_setprio of the entropy waves (0-3; A/B knob)
  int entropy_prio = 0;
  // parse_kernel workgroup size (its marker walk is one thread's)
  int parse_threads = 64;  // (r05 A/B: 64 +1 % over 256 at four lanes)
  int entropy_lds_pad = 0;  // extra (unused) dynamic LDS per entropy workgroup: CU packing
  PlanCache plans;          // swscale plans per distinct geometry
  // skip the event waits that stream order already implies: the workspace's
  // previous batch on the same stream, and a caller stream with nothing
  // pending (r06 A/B, profiles/r06/ab/lean_waits.txt: +0.5-1 %)
  int lean_waits = 1;
  // skip the multi-scan launch of a batch known to hold no multi-scan image
  // (A/B knob; r05: 1 % slower, the empty launch staggered the lanes)
  int ms_skip_empty = 0;
  // XCD-aware tile order (bit 0 sws_kernel, bit 1 idct_kernel): each XCD
  // takes a contiguous range of tiles, so neighbouring bands of an image
  // share their overlapping source rows in one L2 (r06 A/B: mixed 4 lanes
  // +1.4 %, uniform unchanged)
  int xcd_order = 1;
  // piece hand-off wait bound (us of polling with nothing arriving), and the
  // images re-decoded in one workgroup after a wait gave up
  int64_t handoff_wait_us = 2000000;
  int64_t handoff_retries = 0;
};

namespace {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// The copy pool is only needed by host-side packing of large batches; the
// device-resident entry points never create it.
CopyPool* copy_pool(spdl_hj_ctx* c) {
  if (!c->pool) c->pool = new CopyPool(copy_workers());  // + the calling thread
  return c->pool;
}

hipError_t create_stream(hipStream_t* s, int priority) {
  int least = 0, greatest = 0;
  (void)hipDeviceGetStreamPriorityRange(&least, &greatest);  // (1, -1) on gfx950
  return hipStreamCreateWithPriority(s, hipStreamNonBlocking,
                                     std::max(greatest, std::min(least, priority)));
}

// side streams (multiscan beside the lanes' stages) have queues to spare: the
// high-priority pool holds them alone unless the lanes are high priority too
bool side_streams_fit(const spdl_hj_ctx* c) {
  return (c->lane_priority < 0 ? 2 * c->lanes : c->lanes) <= c->hw_queues;
}

// Workspaces [0, n) get their completion event and (n > 1) their stream.
bool ensure_lanes(spdl_hj_ctx* c, int n) {
  DeviceGuard g(c->device);
  for (int i = c->lanes_ready; i < n; i++) {
    Workspace& w = c->ws[i];
    if (!w.done && hipEventCreateWithFlags(&w.done, hipEventDisableTiming) != hipSuccess) return false;
    if (!w.stream && create_stream(&w.stream, c->lane_priority) != hipSuccess) return false;
    c->lanes_ready = i + 1;
  }
  return true;
}

#define HJ_HIP(expr)                                                                     \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess) {                                                              \
      set_err(err, errlen, "HIP error %s at %s:%d (%s)", hipGetErrorString(e_), __FILE__, \
              __LINE__, #expr);                                                          \
      return e_ == hipErrorOutOfMemory ? SPDL_HJ_ERR_OOM : SPDL_HJ_ERR_HIP;             \
    }                                                                                    \
  } while (0)

// stage boundary i: recorded when profiling and a profiled stage starts or
// ends there ("profile_stages": stage i spans ev[i] .. ev[i + 1])
inline void mark(spdl_hj_ctx* c, Slot& s, int i, hipStream_t st) {
  if (c->profiling && ((c->profile_stages | (c->profile_stages << 1)) >> i & 1u))
    (void)hipEventRecord(s.ev[i], st);
}

// Take the next ring slot: its previous batch (if any) must have finished
// before its pinned staging may be rewritten.  An un-waited ticket's
// statuses are dropped here (the ring holds kSlots batches in flight).
int acquire_slot(spdl_hj_ctx* ctx, Slot** out, char* err, size_t errlen) {
  Slot& s = ctx->slots[ctx->next_ticket % kSlots];
  if (s.staged) {
    set_err(err, errlen, "staging slot of ticket %lld was acquired but never submitted",
            (long long)s.ticket);
    return SPDL_HJ_ERR_INVALID_ARG;
  }
  if (s.ticket) HJ_HIP(hipEventSynchronize(s.done));
  s.pending = false;
  s.ticket = ctx->next_ticket++;
  *out = &s;
  return SPDL_HJ_OK;
}

Slot* find_slot(spdl_hj_ctx* ctx, int64_t ticket) {
  if (ticket <= 0) return nullptr;
  Slot& s = ctx->slots[ticket % kSlots];
  return s.ticket == ticket ? &s : nullptr;
}

int retry_image(spdl_hj_ctx* ctx, const Slot::Retry& r, int k);

// Per-image statuses of a finished slot -> status[], first error -> err;
// its stage timings -> ctx->timings when it was profiled.
int collect_status(spdl_hj_ctx* ctx, Slot& s, int32_t* status, char* err, size_t errlen) {
  if (s.profiled) {
    ctx->ntimings = kStages;
    for (int i = 0; i < kStages; i++) {
      float ms = -1.f;  // (stages not profiled, or a failed query: -1)
      if (!(s.profiled_stages >> i & 1u) ||
          hipEventElapsedTime(&ms, s.ev[i], s.ev[i + 1]) != hipSuccess)
        ms = -1.f;
      ctx->timings[i] = ms < 0.f ? -1.f : ms * 1000.f;
    }
    s.profiled = false;
  }
  const int32_t* stv = static_cast<const int32_t*>(s.pin_status.p);
  s.pending = false;
  bool handoff = false;
  for (int i = 0; i < s.n && !handoff; i++) handoff = stv[i] == SPDL_HJ_ERR_HANDOFF;
  std::vector<int32_t> fixed;
  if (handoff && !s.retry.idx.empty()) {
    // re-decode each image whose hand-off gave up in one workgroup (its
    // output lands where the batch's would have; the spare slot, statuses
    // copied first all the same)
    fixed.assign(stv, stv + s.n);
    Slot::Retry r = std::move(s.retry);
    s.retry = Slot::Retry{};
    for (size_t k = 0; k < r.idx.size(); k++)
      if (fixed[r.idx[k]] == SPDL_HJ_ERR_HANDOFF) fixed[r.idx[k]] = retry_image(ctx, r, (int)k);
    stv = fixed.data();
  }
  const int n = fixed.empty() ? s.n : (int)fixed.size();
  int first_bad = -1;
  for (int i = 0; i < n; i++) {
    if (status) status[i] = stv[i];
    if (stv[i] != SPDL_HJ_OK && first_bad < 0) first_bad = i;
  }
  if (first_bad >= 0) {
    set_err(err, errlen, "Failed to decode an image. (image %d: %s)", first_bad,
            status_str(stv[first_bad]));
    return stv[first_bad];
  }
  return SPDL_HJ_OK;
}

// device pipeline over bytes already in HBM; `slot` provides the descriptor
// and status staging and is marked done on `st` at the end.  `st` is the
// execution stream (exec_stream()), the workspace is the slot's lane.
int run_pipeline(spdl_hj_ctx* ctx, Slot& slot, const uint8_t* d_bytes, size_t bytes_len,
                 const Layout& L, int n, const spdl_hj_output* out, void* out_dev,
                 size_t out_bytes, hipStream_t st, int sync, int32_t* status, char* err,
                 size_t errlen, bool planes_only) {
  const size_t esz = out->dtype == SPDL_HJ_DTYPE_U8 ? 1 : 2;
  if (!planes_only && (size_t)L.out_elems_per_image * n * esz > out_bytes) {
    set_err(err, errlen, "output buffer too small: need %lld bytes, have %zu",
            (long long)(L.out_elems_per_image * n * esz), out_bytes);
    return SPDL_HJ_ERR_INVALID_ARG;
  }
  int64_t max_end = 0;
  for (int i = 0; i < n; i++) {
    if (L.desc[i].in_off % 256) {
      set_err(err, errlen, "image %d offset %lld is not 256-byte aligned", i,
              (long long)L.desc[i].in_off);
      return SPDL_HJ_ERR_INVALID_ARG;
    }
    int64_t e = L.desc[i].in_off + L.desc[i].in_size;
    if (L.desc[i].in_off < 0 || L.desc[i].in_size < 0 || (size_t)e > bytes_len) {
      set_err(err, errlen, "image %d extends past the input buffer", i);
      return SPDL_HJ_ERR_INVALID_ARG;
    }
    if (e > max_end) max_end = e;
  }
  Workspace& W = ctx->ws[slot.ticket % ctx->lanes];
  // the previous batch may still be using the workspace (async call, maybe on
  // another stream; on the same stream, stream order already covers it)
  if (!(ctx->lean_waits && W.used && W.last_st == st)) HJ_HIP(hipStreamWaitEvent(st, W.done, 0));
  W.last_st = st;
  W.used = true;
  HJ_HIP(W.clean.ensure((size_t)max_end + 512, st, true));
  HJ_HIP(W.segs.ensure((size_t)L.total_segs * 4 + 64, st, true));
  HJ_HIP(W.dschunks.ensure((size_t)L.total_ds * sizeof(DsChunk) + 64, st, true));
  const int nwork = (int)L.work.size();
  const size_t desc_bytes = sizeof(ImageDesc) * n + sizeof(uint32_t) * nwork;  // + work list
  HJ_HIP(W.desc.ensure(desc_bytes, st, true));
  HJ_HIP(W.chain.ensure((size_t)(kChainHead + L.chain_granules) * 8 + 64, st, true));
  HJ_HIP(W.maps.ensure((size_t)(L.ds_wgs + L.idct_wgs + L.hs_wgs + L.sws_wgs) * 4 + 64, st, true));
  HJ_HIP(W.hbuf.ensure((size_t)L.total_hbuf * 2 + 64, st, true));
  auto* ds_map = static_cast<uint32_t*>(W.maps.p);
  auto* idct_map = ds_map + L.ds_wgs;
  auto* hs_map = idct_map + L.idct_wgs;
  auto* sws_map = hs_map + L.hs_wgs;
  // A grid is flat (one workgroup per image tile, through the map) when the
  // (max tiles) x images grid would be mostly empty; a batch of similar
  // images keeps the 2-D grid, whose workgroups need no map lookup
  auto use_flat = [&](int64_t flat_wgs, int64_t max_tiles) {
    return (double)max_tiles * n > 1.25 * (double)flat_wgs;
  };
  const bool ds_flat = use_flat(L.ds_wgs, L.max_chunks);
  const bool idct_flat = use_flat(L.idct_wgs, (L.max_blocks + kIdctThreads - 1) / kIdctThreads);
  const bool sws_flat = use_flat(L.sws_wgs, (int64_t)L.sws_bands * L.sws_chunks);
  HJ_HIP(W.info.ensure(sizeof(ImageInfo) * n, st, true));
  HJ_HIP(W.luts.ensure(sizeof(HuffTable) * 8 * n, st, true));
  HJ_HIP(W.ents.ensure((size_t)L.total_blocks * 256 + 256, st, true));
  HJ_HIP(W.bdesc.ensure((size_t)L.total_blocks * 8 + 64, st, true));
  HJ_HIP(W.planes.ensure((size_t)L.total_planes + 256, st, true));
  HJ_HIP(W.recs.ensure((size_t)L.total_recs * 4 + 256, st, true));
  HJ_HIP(W.wts.ensure(L.tables.size() * 4 + 256, st, true));
  HJ_HIP(slot.pin_desc.ensure(desc_bytes));
  HJ_HIP(slot.pin_status.ensure(sizeof(int32_t) * n));
  slot.n = n;
  memcpy(slot.pin_desc.p, L.desc.data(), sizeof(ImageDesc) * n);
  memcpy(static_cast<ImageDesc*>(slot.pin_desc.p) + n, L.work.data(), sizeof(uint32_t) * nwork);
  // the batch's swscale tables travel with the descriptors
  const bool swscale = !planes_only && out->csc == SPDL_HJ_CSC_SWSCALE;
  const size_t tb = swscale ? L.tables.size() * 4 : 0;
  HJ_HIP(slot.pin_tables.ensure(tb + 16));
  if (tb) memcpy(slot.pin_tables.p, L.tables.data(), tb);
  const bool hs = ctx->host_staging != 0;
  if (!hs) {
    HJ_HIP(hipMemcpyAsync(W.desc.p, slot.pin_desc.p, desc_bytes, hipMemcpyHostToDevice, st));
    if (tb) HJ_HIP(hipMemcpyAsync(W.wts.p, slot.pin_tables.p, tb, hipMemcpyHostToDevice, st));
  }
  mark(ctx, slot, 1, st);
  auto* desc = static_cast<const ImageDesc*>(W.desc.p);
  auto* infos = static_cast<ImageInfo*>(W.info.p);
  auto* work = reinterpret_cast<uint32_t*>(static_cast<ImageDesc*>(W.desc.p) + n);
  auto* chain = static_cast<uint64_t*>(W.chain.p);
  HJ_HIP(launch_parse(d_bytes, hs ? static_cast<const ImageDesc*>(slot.pin_desc.dev) : nullptr,
                      static_cast<ImageDesc*>(W.desc.p), infos,
                      static_cast<HuffTable*>(W.luts.p), hs ? slot.pin_tables.dev : nullptr,
                      W.wts.p, hs ? (int64_t)tb : 0,
                      hs ? reinterpret_cast<const uint32_t*>(
                               static_cast<const ImageDesc*>(slot.pin_desc.dev) + n)
                         : nullptr,
                      work, nwork, chain, ds_map, idct_map, hs_map, sws_map, ctx->parse_threads, n,
                      st));
  mark(ctx, slot, 2, st);
  const bool ms_side = L.ms_side && !(ctx->debug_mask & 0x10000) && side_streams_fit(ctx);
  if (ms_side) {
    if (!W.side) HJ_HIP(create_stream(&W.side, -1));
    if (!W.ev_parsed) HJ_HIP(hipEventCreateWithFlags(&W.ev_parsed, hipEventDisableTiming));
    if (!W.ev_ms) HJ_HIP(hipEventCreateWithFlags(&W.ev_ms, hipEventDisableTiming));
    HJ_HIP(hipEventRecord(W.ev_parsed, st));
    HJ_HIP(hipStreamWaitEvent(W.side, W.ev_parsed, 0));
    HJ_HIP(launch_multiscan(d_bytes, static_cast<uint8_t*>(W.clean.p), desc, infos,
                            static_cast<uint32_t*>(W.ents.p), static_cast<uint2*>(W.bdesc.p), n,
                            W.side));
    HJ_HIP(hipEventRecord(W.ev_ms, W.side));
  }
  // If a launch below fails and returns early, the lane's stream still joins
  // the side stream and re-records W.done, so the next batch on this
  // workspace cannot reuse clean / ents / bdesc while multiscan writes them.
  struct SideJoin {
    hipStream_t st = nullptr;
    Workspace* w = nullptr;
    ~SideJoin() {
      if (!w) return;
      (void)hipStreamWaitEvent(st, w->ev_ms, 0);
      (void)hipEventRecord(w->done, st);
    }
  } side_join;
  if (ms_side) {
    side_join.st = st;
    side_join.w = &W;
  }
  HJ_HIP(launch_destuff(d_bytes, desc, infos, static_cast<DsChunk*>(W.dschunks.p),
                        static_cast<uint8_t*>(W.clean.p), static_cast<uint32_t*>(W.segs.p),
                        ds_flat ? ds_map : nullptr, (int)L.ds_wgs, L.max_chunks, n, st));
  mark(ctx, slot, 3, st);
  const int ent_threads =
      ctx->entropy_threads ? ctx->entropy_threads : (ctx->lanes > 1 ? 256 : 512);
  const int warm = ctx->warm_slots >= 0 ? ctx->warm_slots : (ent_threads <= 256 ? 6 : 12);
  HJ_HIP(launch_entropy(static_cast<const uint8_t*>(W.clean.p),
                        static_cast<const uint32_t*>(W.segs.p), desc, infos,
                        static_cast<const HuffTable*>(W.luts.p),
                        static_cast<uint32_t*>(W.ents.p), static_cast<uint2*>(W.bdesc.p),
                        static_cast<uint32_t*>(W.recs.p), work, chain,
                        ctx->sub_bits,
                        warm | (ctx->min_run_slots << 8) |
                            ((ctx->chain_after >= 0 ? ctx->chain_after : (ent_threads >= 512 ? 1 : 2))
                             << 26) |
                            ((((ctx->debug_mask >> 12) & 0xF) | (((ctx->debug_mask >> 19) & 1) << 4))
                             << 16) |
                            (ctx->entropy_prio << 24),
                        ent_threads, ctx->entropy_lds_pad, nwork, ctx->handoff_wait_us * 100, st));
  // (the entropy stage ends here: the multiscan launch or the wait for the
  // side stream counts to the IDCT stage)
  mark(ctx, slot, 4, st);
  // progressive / non-interleaved images (the kernels above skipped them)
  // (debug_mask 0x10000 / 0x20000 / 0x40000: timing ablations that skip the
  // multiscan / IDCT / output launch; the output is wrong)
  if (ms_side) {
    side_join.w = nullptr;
    HJ_HIP(hipStreamWaitEvent(st, W.ev_ms, 0));
  } else if (!(ctx->debug_mask & 0x10000) && !(ctx->ms_skip_empty && L.ms_known && !L.ms_side))
    HJ_HIP(launch_multiscan(d_bytes, static_cast<uint8_t*>(W.clean.p), desc, infos,
                            static_cast<uint32_t*>(W.ents.p),
                            static_cast<uint2*>(W.bdesc.p), n, st));
  // full resolution u8 through swscale's unscaled converter: IDCT and
  // conversion in one kernel (output_path 1: the generic sws_kernel, 2:
  // separate IDCT + rgb_unscaled_kernel)
  const int idct_kind = (ctx->debug_mask & 0x800) ? 2 : out->idct;
  const bool fast_rgb = swscale && L.all_special && out->dtype == SPDL_HJ_DTYPE_U8 &&
                        ctx->output_path != 1;
  const bool fused = fast_rgb && L.fuse_ok && L.fused_tiles > 0 && ctx->output_path != 2;
  if (!(ctx->debug_mask & 0x20000) && !fused)
    HJ_HIP(launch_idct(static_cast<const uint32_t*>(W.ents.p),
                     static_cast<const uint2*>(W.bdesc.p), desc, infos,
                     static_cast<uint8_t*>(W.planes.p), idct_kind, idct_flat ? idct_map : nullptr,
                     (int)L.idct_wgs, L.max_blocks, n, (ctx->xcd_order >> 1) & 1, st));
  // 4-component frames: FFmpeg's K transform on the planes (not on the raw
  // planes surface, which returns the IDCT output as the oracle does)
  if (!planes_only && L.cmyk_px > 0)
    HJ_HIP(launch_cmyk(desc, infos, static_cast<uint8_t*>(W.planes.p), L.cmyk_px, n, st));
  mark(ctx, slot, 5, st);
  BatchParams bp{};
  bp.n = n;
  bp.pix_fmt = out->pix_fmt;
  bp.dtype = out->dtype;
  bp.idct = out->idct;
  bp.resize = out->resize;
  bp.filter = out->filter;
  bp.out_w = L.ow;
  bp.out_h = L.oh;
  bp.sub_bits = ctx->sub_bits;
  bp.debug_mask = ctx->debug_mask;
  bp.xcd_order = ctx->xcd_order;
  for (int c = 0; c < 3; c++) {
    bp.mean[c] = out->mean[c];
    bp.std[c] = out->std[c];
  }
  const SwsCsc csc = sws_csc();
  bp.crv = csc.crv;
  bp.cbu = csc.cbu;
  bp.cgu = csc.cgu;
  bp.cgv = csc.cgv;
  bp.y_coeff = csc.y_coeff;
  bp.y_offset = csc.y_offset;
  bp.v2r = csc.v2r;
  bp.v2g = csc.v2g;
  bp.u2g = csc.u2g;
  bp.u2b = csc.u2b;
  // the output kernel writes each image's status into the pinned array itself
  int32_t* hstat = hs && !planes_only ? static_cast<int32_t*>(slot.pin_status.dev) : nullptr;
  mark(ctx, slot, 6, st);
  if (!planes_only && !(ctx->debug_mask & 0x40000)) {
    if (fused) {
      HJ_HIP(launch_idct_rgb(static_cast<const uint32_t*>(W.ents.p),
                             static_cast<const uint2*>(W.bdesc.p), desc, infos, out_dev, bp,
                             idct_kind, L.fused_tiles, n, hstat, st));
    } else if (fast_rgb) {
      // full resolution, u8: swscale's unscaled converter needs no scaling passes
      HJ_HIP(launch_rgb_unscaled(static_cast<const uint8_t*>(W.planes.p), desc, infos, out_dev,
                                 bp, L.max_px, n, hstat, st));
    } else if (swscale) {
      HJ_HIP(launch_sws(static_cast<const uint8_t*>(W.planes.p), desc, infos,
                        static_cast<const int32_t*>(W.wts.p), out_dev, bp,
                        sws_flat ? sws_map : nullptr, (int)L.sws_wgs, L.sws_bands, L.sws_chunks, n,
                        L.sws_lds, hstat, hs_map, (int)L.hs_wgs,
                        static_cast<int16_t*>(W.hbuf.p), st));
    } else {
      HJ_HIP(launch_csc(static_cast<const uint8_t*>(W.planes.p), desc, infos, out_dev, bp,
                        L.max_px, n, hstat, st));
    }
  }
  mark(ctx, slot, 7, st);
  // per-image status: strided D2H of ImageInfo::status
  if (!hstat)
    HJ_HIP(hipMemcpy2DAsync(slot.pin_status.p, sizeof(int32_t), W.info.p, sizeof(ImageInfo),
                            sizeof(int32_t), n, hipMemcpyDeviceToHost, st));
  mark(ctx, slot, 8, st);
  HJ_HIP(hipEventRecord(W.done, st));
  HJ_HIP(hipEventRecord(slot.done, st));
  Slot::Retry& R = slot.retry;
  R.idx.clear();
  R.off.clear();
  R.size.clear();
  R.info.clear();
  if (!planes_only) {
    for (const auto& m : L.multi) {
      R.idx.push_back(m.first);
      R.off.push_back(L.desc[m.first].in_off);
      R.size.push_back(L.desc[m.first].in_size);
      R.info.push_back(m.second);
    }
    R.ticket = slot.ticket;
    R.bytes = d_bytes;
    R.len = bytes_len;
    R.out = *out;
    R.out_dev = static_cast<uint8_t*>(out_dev);
    R.img_bytes = (size_t)L.out_elems_per_image * esz;
  }
  slot.pending = true;
  slot.profiled = ctx->profiling;
  slot.profiled_stages = ctx->profile_stages;
  ctx->last_ticket = slot.ticket;
  if (!sync) return SPDL_HJ_OK;
  HJ_HIP(hipEventSynchronize(slot.done));
  return collect_status(ctx, slot, status, err, errlen);
}

// Stream the batch of `slot` executes on: the caller's stream with one lane;
// otherwise its lane's own stream, ordered after everything the caller's
// stream has queued so far (its output allocation, say).  Completion is then
// observed through the ticket (spdl_hj_wait / spdl_hj_stream_wait), not by
// the caller's stream.
int exec_stream(spdl_hj_ctx* ctx, Slot& slot, hipStream_t st, hipStream_t* xs, char* err,
                size_t errlen) {
  if (ctx->lanes <= 1) {
    *xs = st;
    return SPDL_HJ_OK;
  }
  Workspace& W = ctx->ws[slot.ticket % ctx->lanes];
  // (a caller stream with nothing pending orders nothing: no cross-queue wait.
  // Not asked of the null / per-thread default streams: a query of the
  // legacy null stream waits for the device's other blocking streams -- a
  // test with a GEMM loop on a torch side stream saw every decode wait for it)
  const bool special = st == nullptr || st == hipStreamPerThread;
  if (!(ctx->lean_waits && !special && hipStreamQuery(st) == hipSuccess)) {
    HJ_HIP(hipEventRecord(slot.submitted, st));
    HJ_HIP(hipStreamWaitEvent(W.stream, slot.submitted, 0));
  }
  *xs = W.stream;
  return SPDL_HJ_OK;
}

// Image r.idx[k] of a finished batch again, as a one-image batch decoded by
// one entropy workgroup (no piece hand-off), synchronously, into its place in
// the batch's output.  Returns its status.
int retry_image(spdl_hj_ctx* ctx, const Slot::Retry& r, int k) {
  char err[256];
  const size_t errlen = sizeof(err);
  Layout L;
  int32_t st1 = SPDL_HJ_OK;
  int rc = build_layout(&r.off[k], &r.size[k], &r.info[k], 1, &r.out, ctx->sub_bits, 0, L, &st1,
                        err, errlen, &ctx->plans);
  if (rc) return rc;
  // the spare slot, on the failed batch's lane (its workspace is free: the
  // batch has finished); the caller's last ticket is left as it was
  Slot* s = &ctx->slots[kSlots];
  if (s->ticket && hipEventSynchronize(s->done) != hipSuccess) return SPDL_HJ_ERR_HIP;
  s->ticket = r.ticket;
  s->pending = false;
  const int64_t last = ctx->last_ticket;
  hipStream_t xs;
  rc = exec_stream(ctx, *s, nullptr, &xs, err, errlen);
  if (rc) return rc;
  ctx->handoff_retries++;
  rc = run_pipeline(ctx, *s, r.bytes, r.len, L, 1, &r.out, r.out_dev + (size_t)r.idx[k] * r.img_bytes,
                    r.img_bytes, xs, 1, &st1, err, errlen, false);
  ctx->last_ticket = last;
  return rc ? rc : st1;
}

// H2D of the slot's staged bytes on the copy stream; `st` waits for it.
int stage_h2d(spdl_hj_ctx* ctx, Slot& s, size_t total, hipStream_t st, char* err, size_t errlen) {
  // (created on first use: device-resident batches never take its queue)
  if (!ctx->copy) HJ_HIP(hipStreamCreateWithFlags(&ctx->copy, hipStreamNonBlocking));
  // (the slot's previous batch has finished: acquire_slot waited for it)
  HJ_HIP(s.bytes.ensure(total + 512, ctx->copy, true));
  mark(ctx, s, 0, ctx->copy);
  HJ_HIP(hipMemcpyAsync(s.bytes.p, s.pin_in.p, total, hipMemcpyHostToDevice, ctx->copy));
  HJ_HIP(hipEventRecord(s.h2d_done, ctx->copy));
  HJ_HIP(hipStreamWaitEvent(st, s.h2d_done, 0));
  return SPDL_HJ_OK;
}

bool valid_output(const spdl_hj_output* o) {
  // the JFIF conversion has no scaler: full resolution only
  return o && o->pix_fmt >= 0 && o->pix_fmt <= 3 && (o->dtype >= 0 && o->dtype <= 2) &&
         (o->idct == 0 || o->idct == 1) && (o->filter >= 0 && o->filter <= 2) &&
         o->aspect >= 0 && o->aspect <= 2 &&
         (o->csc == SPDL_HJ_CSC_SWSCALE || (o->csc == SPDL_HJ_CSC_JFIF && !o->resize));
}

// ---- tar (ustar / GNU 'L' long names / pax 'x' path) ------------------------
// Same member walk as the reference's InMemoryTarParserImpl::parse_next
// (src/spdl/io/lib/archive/tar_iterator.cpp:125-195): a header that fails the
// magic/checksum test is skipped 512 bytes at a time; an empty name ends the
// archive; 'L' and 'x' records name the next regular file; other types are
// skipped with their payload; a member running past the buffer ends the walk.
uint64_t tar_octal(const uint8_t* s, size_t n) {
  uint64_t r = 0;
  for (size_t i = 0; i < n && s[i] != 0 && s[i] != ' '; i++)
    if (s[i] >= '0' && s[i] <= '7') r = r * 8 + (s[i] - '0');
  return r;
}

bool tar_header_ok(const uint8_t* h) {
  if (memcmp(h + 257, "ustar", 5) != 0) return false;
  uint32_t sum = 0;
  for (int i = 0; i < 512; i++) sum += (i >= 148 && i < 156) ? (uint32_t)' ' : h[i];
  return tar_octal(h + 148, 8) == sum;
}

std::string tar_pax_path(const uint8_t* d, size_t n) {
  // records "<len> key=value\n"
  size_t pos = 0;
  while (pos < n) {
    const void* sp = memchr(d + pos, ' ', n - pos);
    if (!sp) break;
    const size_t rs = (size_t)(static_cast<const uint8_t*>(sp) - d) + 1;
    if (rs + 5 <= n && memcmp(d + rs, "path=", 5) == 0) {
      const void* nl = memchr(d + rs + 5, '\n', n - rs - 5);
      if (nl) return std::string((const char*)d + rs + 5,
                                 (size_t)(static_cast<const uint8_t*>(nl) - (d + rs + 5)));
    }
    const void* nl = memchr(d + pos, '\n', n - pos);
    if (!nl) break;
    pos = (size_t)(static_cast<const uint8_t*>(nl) - d) + 1;
  }
  return std::string();
}

}  // namespace

extern "C" {

int spdl_hj_abi_version(void) { return SPDL_HJ_ABI_VERSION; }

int spdl_hj_get_image_info(const uint8_t* data, size_t size, spdl_hj_image_info* info) {
  if (!info) return SPDL_HJ_ERR_INVALID_ARG;
  return probe(data, size, info);
}

int spdl_hj_output_size(int32_t w, int32_t h, const spdl_hj_output* out, int32_t* out_w,
                        int32_t* out_h) {
  if (!valid_output(out) || !out_w || !out_h) return SPDL_HJ_ERR_INVALID_ARG;
  Geom g;
  int rc = geometry(w, h, out, &g);
  if (rc) return rc;
  *out_w = g.ow;
  *out_h = g.oh;
  return SPDL_HJ_OK;
}

spdl_hj_ctx* spdl_hj_create(int device, char* err, size_t errlen) {
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count <= 0) {
    set_err(err, errlen, "no HIP device available (%s)", hipGetErrorString(e));
    return nullptr;
  }
  if (device < 0 || device >= count) {
    set_err(err, errlen, "device index %d out of range (%d devices)", device, count);
    return nullptr;
  }
  DeviceGuard g(device);
  auto* c = new spdl_hj_ctx();
  c->device = device;
  if (const char* q = getenv("GPU_MAX_HW_QUEUES")) c->hw_queues = atoi(q) > 0 ? atoi(q) : 4;
  bool ok = ensure_lanes(c, 1);
  for (int i = 0; ok && i <= kSlots; i++)
    ok = hipEventCreateWithFlags(&c->slots[i].h2d_done, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&c->slots[i].done, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&c->slots[i].submitted, hipEventDisableTiming) == hipSuccess;
  for (int i = 0; ok && i <= kSlots; i++)
    for (int k = 0; ok && k <= kStages; k++) ok = hipEventCreate(&c->slots[i].ev[k]) == hipSuccess;
  if (!ok) {
    set_err(err, errlen, "hipEventCreate / hipStreamCreate failed");
    spdl_hj_destroy(c);
    return nullptr;
  }
  return c;
}

void spdl_hj_destroy(spdl_hj_ctx* c) {
  if (!c) return;
  DeviceGuard g(c->device);
  for (Slot& s : c->slots)
    if (s.ticket && s.done) (void)hipEventSynchronize(s.done);
  for (Workspace& w : c->ws) {
    if (w.done) (void)hipEventSynchronize(w.done);
    if (w.stream) (void)hipStreamSynchronize(w.stream);
  }
  if (c->copy) (void)hipStreamSynchronize(c->copy);
  for (Workspace& w : c->ws) {
    DevBuf* bufs[] = {&w.clean, &w.segs, &w.desc, &w.info, &w.luts, &w.ents, &w.bdesc,
                      &w.planes, &w.wts, &w.recs, &w.dschunks};
    for (DevBuf* b : bufs) b->release();
    if (w.done) (void)hipEventDestroy(w.done);
    if (w.stream) (void)hipStreamDestroy(w.stream);
    if (w.ev_parsed) (void)hipEventDestroy(w.ev_parsed);
    if (w.ev_ms) (void)hipEventDestroy(w.ev_ms);
    if (w.side) (void)hipStreamDestroy(w.side);
  }
  for (Slot& s : c->slots) {
    s.bytes.release();
    s.pin_in.release();
    s.pin_desc.release();
    s.pin_status.release();
    s.pin_tables.release();
    if (s.h2d_done) (void)hipEventDestroy(s.h2d_done);
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.submitted) (void)hipEventDestroy(s.submitted);
    for (int k = 0; k <= kStages; k++)
      if (s.ev[k]) (void)hipEventDestroy(s.ev[k]);
  }
  if (c->copy) (void)hipStreamDestroy(c->copy);
  delete c->pool;
  delete c;
}

int spdl_hj_decode_batch(spdl_hj_ctx* ctx, const uint8_t* const* data, const size_t* sizes,
                         int32_t n, const spdl_hj_output* out, void* out_dev, size_t out_bytes,
                         void* stream, int32_t sync, int32_t* status, char* err, size_t errlen) {
  if (!ctx || !data || !sizes || n <= 0 || !valid_output(out) || !out_dev) {
    set_err(err, errlen, n <= 0 ? "the batch is empty" : "invalid argument");
    return SPDL_HJ_ERR_INVALID_ARG;
  }
  DeviceGuard g(ctx->device);
  hipStream_t st = static_cast<hipStream_t>(stream);
  std::vector<spdl_hj_image_info> infos(n);
  std::vector<int64_t> offs(n), szs(n);
  std::vector<CopyItem> items(n);
  int64_t total = 0;
  bool prog = false;
  for (int i = 0; i < n; i++) {
    int rc = probe(data[i], sizes[i], &infos[i]);
    if (!rc) prog = prog || infos[i].multiscan;
    if (status) status[i] = rc;
    if (rc) {
      set_err(err, errlen, "Failed to decode an image. (image %d: %s)", i, status_str(rc));
      return rc;
    }
    offs[i] = total;
    szs[i] = (int64_t)sizes[i];
    const int64_t padded = round_up((int64_t)sizes[i] + 64, 256);
    items[i] = {total, data[i], (int64_t)sizes[i], padded};
    total += padded;
  }
  Layout L;
  int rc = build_layout(offs.data(), szs.data(), infos.data(), n, out, ctx->sub_bits, ctx->piece_bytes, L, status, err,
                        errlen, &ctx->plans);
  if (rc) return rc;
  L.ms_side = prog;
  L.ms_known = true;
  Slot* s = nullptr;
  rc = acquire_slot(ctx, &s, err, errlen);
  if (rc) return rc;
  HJ_HIP(s->pin_in.ensure((size_t)total));
  parallel_pack(copy_pool(ctx), static_cast<uint8_t*>(s->pin_in.p), items);
  hipStream_t xs;
  rc = exec_stream(ctx, *s, st, &xs, err, errlen);
  if (!rc) rc = stage_h2d(ctx, *s, (size_t)total, xs, err, errlen);
  if (rc) return rc;
  return run_pipeline(ctx, *s, static_cast<const uint8_t*>(s->bytes.p), (size_t)total, L, n, out,
                      out_dev, out_bytes, xs, sync, status, err, errlen, false);
}

int spdl_hj_decode_batch_device(spdl_hj_ctx* ctx, const uint8_t* dev_data, size_t dev_bytes,
                                const int64_t* offsets, const int64_t* sizes,
                                const spdl_hj_image_info* infos, int32_t n,
                                const spdl_hj_output* out, void* out_dev, size_t out_bytes,
                                void* stream, int32_t sync, int32_t* status, char* err,
                                size_t errlen) {
  if (!ctx || !dev_data || !offsets || !sizes || !infos || n <= 0 || !valid_output(out) ||
      !out_dev) {
    set_err(err, errlen, n <= 0 ? "the batch is empty" : "invalid argument");
    return SPDL_HJ_ERR_INVALID_ARG;
  }
  DeviceGuard g(ctx->device);
  hipStream_t st = static_cast<hipStream_t>(stream);
  Layout L;
  int rc = build_layout(offsets, sizes, infos, n, out, ctx->sub_bits, ctx->piece_bytes, L, status, err, errlen,
                        &ctx->plans);
  if (rc) return rc;
  // the caller's probe says which files take the multi-scan path (ABI 5)
  for (int i = 0; i < n; i++) L.ms_side = L.ms_side || infos[i].multiscan != 0;
  L.ms_known = true;
  Slot* s = nullptr;
  rc = acquire_slot(ctx, &s, err, errlen);
  if (rc) return rc;
  hipStream_t xs;
  rc = exec_stream(ctx, *s, st, &xs, err, errlen);
  if (rc) return rc;
  mark(ctx, *s, 0, xs);
  return run_pipeline(ctx, *s, dev_data, dev_bytes, L, n, out, out_dev, out_bytes, xs, sync,
                      status, err, errlen, false);
}

int64_t spdl_hj_last_ticket(spdl_hj_ctx* ctx) { return ctx ? ctx->last_ticket : 0; }

int spdl_hj_wait(spdl_hj_ctx* ctx, int64_t ticket, int32_t* status, int32_t n, char* err,
                 size_t errlen) {
  if (!ctx) return SPDL_HJ_ERR_INVALID_ARG;
  Slot* s = find_slot(ctx, ticket);
  if (!s || !s->pending) {
    set_err(err, errlen, "unknown, already waited or overwritten ticket %lld", (long long)ticket);
    return SPDL_HJ_ERR_INVALID_ARG;
  }
  if (status && n < s->n) {
    set_err(err, errlen, "status array too small (%d < %d)", n, s->n);
    return SPDL_HJ_ERR_INVALID_ARG;
  }
  DeviceGuard g(ctx->device);
  HJ_HIP(hipEventSynchronize(s->done));
  return collect_status(ctx, *s, status, err, errlen);
}

int spdl_hj_stream_wait(spdl_hj_ctx* ctx, int64_t ticket, void* stream, char* err,
                        size_t errlen) {
  Slot* s = ctx ? find_slot(ctx, ticket) : nullptr;
  if (!s) {
    set_err(err, errlen, "unknown or overwritten ticket %lld", (long long)ticket);
    return SPDL_HJ_ERR_INVALID_ARG;
  }
  DeviceGuard g(ctx->device);
  HJ_HIP(hipStreamWaitEvent(static_cast<hipStream_t>(stream), s->done, 0));
  return SPDL_HJ_OK;
}

int spdl_hj_staging_acquire(spdl_hj_ctx* ctx, size_t bytes, uint8_t** host_ptr, int64_t* ticket,
                            char* err, size_t errlen) {
  if (!ctx || !host_ptr || !ticket) {
    set_err(err, errlen, "invalid argument");
    return SPDL_HJ_ERR_INVALID_ARG;
  }
  DeviceGuard g(ctx->device);
  Slot* s = nullptr;
  int rc = acquire_slot(ctx, &s, err, errlen);
  if (rc) return rc;
  HJ_HIP(s->pin_in.ensure(bytes + 512));
  s->staged = true;
  *host_ptr = static_cast<uint8_t*>(s->pin_in.p);
  *ticket = s->ticket;
  return SPDL_HJ_OK;
}

int spdl_hj_staging_fill(spdl_hj_ctx* ctx, int64_t ticket, size_t dst_off, const uint8_t* src,
                         size_t len, char* err, size_t errlen) {
  Slot* s = ctx ? find_slot(ctx, ticket) : nullptr;
  if (!s || !s->staged || !src || dst_off + len > s->pin_in.cap) {
    set_err(err, errlen, "invalid staging fill (ticket %lld)", (long long)ticket);
    return SPDL_HJ_ERR_INVALID_ARG;
  }
  std::vector<CopyItem> items(1, CopyItem{(int64_t)dst_off, src, (int64_t)len, (int64_t)len});
  parallel_pack(copy_pool(ctx), static_cast<uint8_t*>(s->pin_in.p), items);
  return SPDL_HJ_OK;
}

int spdl_hj_staging_read(spdl_hj_ctx* ctx, int64_t ticket, size_t dst_off, int fd,
                         int64_t file_off, size_t len, char* err, size_t errlen) {
  Slot* s = ctx ? find_slot(ctx, ticket) : nullptr;
  if (!s || !s->staged || fd < 0 || file_off < 0 || dst_off + len > s->pin_in.cap) {
    set_err(err, errlen, "invalid staging read (ticket %lld)", (long long)ticket);
    return SPDL_HJ_ERR_INVALID_ARG;
  }
  uint8_t* base = static_cast<uint8_t*>(s->pin_in.p) + dst_off;
  std::atomic<int> bad{0};
  auto body = [&](int part, int np) {
    // 64 KiB-aligned split so the page-cache copies stay sequential per thread
    const size_t unit = 1 << 16, nu = (len + unit - 1) / unit;
    size_t lo = nu * part / np * unit, hi = nu * (part + 1) / np * unit;
    if (hi > len) hi = len;
    while (lo < hi) {
      const ssize_t r = pread(fd, base + lo, hi - lo, (off_t)(file_off + (int64_t)lo));
      if (r <= 0) {
        bad = 1;
        return;
      }
      lo += (size_t)r;
    }
  };
  if (len < (4u << 20) || copy_pool(ctx)->workers() < 2) body(0, 1);
  else copy_pool(ctx)->run(body);
  if (bad) {
    set_err(err, errlen, "pread failed or hit end of file (offset %lld, %zu bytes)",
            (long long)file_off, len);
    return SPDL_HJ_ERR_INVALID_ARG;
  }
  return SPDL_HJ_OK;
}

int spdl_hj_decode_staged(spdl_hj_ctx* ctx, int64_t ticket, size_t len, const int64_t* offsets,
                          const int64_t* sizes, int32_t n, const spdl_hj_output* out,
                          void* out_dev, size_t out_bytes, void* stream, int32_t sync,
                          int32_t* status, char* err, size_t errlen) {
  Slot* s = ctx ? find_slot(ctx, ticket) : nullptr;
  if (!s || !s->staged) {
    set_err(err, errlen, "ticket %lld does not name an acquired staging slot", (long long)ticket);
    return SPDL_HJ_ERR_INVALID_ARG;
  }
  s->staged = false;  // the slot is consumed whatever happens below
  if (!offsets || !sizes || n <= 0 || !valid_output(out) || !out_dev || len + 512 > s->pin_in.cap) {
    set_err(err, errlen, n <= 0 ? "the batch is empty" : "invalid argument");
    s->ticket = 0;
    return SPDL_HJ_ERR_INVALID_ARG;
  }
  DeviceGuard g(ctx->device);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const uint8_t* host = static_cast<const uint8_t*>(s->pin_in.p);
  std::vector<spdl_hj_image_info> infos(n);
  bool prog = false;
  for (int i = 0; i < n; i++) {
    int rc = SPDL_HJ_ERR_INVALID_ARG;
    if (offsets[i] >= 0 && sizes[i] >= 0 && (size_t)(offsets[i] + sizes[i]) <= len)
      rc = probe(host + offsets[i], (size_t)sizes[i], &infos[i]);
    if (!rc) prog = prog || infos[i].multiscan;
    if (status) status[i] = rc;
    if (rc) {
      set_err(err, errlen, "Failed to decode an image. (image %d: %s)", i, status_str(rc));
      s->ticket = 0;
      return rc;
    }
  }
  Layout L;
  int rc = build_layout(offsets, sizes, infos.data(), n, out, ctx->sub_bits, ctx->piece_bytes, L, status, err, errlen,
                        &ctx->plans);
  if (rc) {
    s->ticket = 0;
    return rc;
  }
  L.ms_side = prog;
  L.ms_known = true;
  memset(static_cast<uint8_t*>(s->pin_in.p) + len, 0, 512);  // tail read slack
  hipStream_t xs;
  rc = exec_stream(ctx, *s, st, &xs, err, errlen);
  if (!rc) rc = stage_h2d(ctx, *s, len + 512, xs, err, errlen);
  if (rc) return rc;
  return run_pipeline(ctx, *s, static_cast<const uint8_t*>(s->bytes.p), len + 512, L, n, out,
                      out_dev, out_bytes, xs, sync, status, err, errlen, false);
}

int spdl_hj_tar_index(const uint8_t* data, size_t size, size_t start, int32_t max_entries,
                      int64_t* offsets, int64_t* sizes, int64_t* name_offs, char* names,
                      size_t names_cap, int32_t* n_out, size_t* next_pos) {
  if (!data || !offsets || !sizes || !n_out || !next_pos || max_entries < 0)
    return SPDL_HJ_ERR_INVALID_ARG;
  size_t pos = start, used = 0;
  int32_t n = 0;
  std::string pending;
  bool at_end = false;
  while (n < max_entries) {
    const size_t entry_pos = pos;  // resume point if this entry does not fit
    std::string path;
    bool found = false;
    pending.clear();
    while (pos + 512 <= size) {
      const uint8_t* h = data + pos;
      if (!tar_header_ok(h)) {
        pos += 512;
        continue;
      }
      std::string fp;
      if (h[0]) {
        if (h[345]) {
          fp.assign((const char*)h + 345, strnlen((const char*)h + 345, 155));
          if (fp.back() != '/') fp += '/';
        }
        fp.append((const char*)h, strnlen((const char*)h, 100));
      }
      if (fp.empty() && pending.empty()) {
        at_end = true;
        break;
      }
      const uint64_t fsz = tar_octal(h + 124, 12);
      const uint64_t padded = (fsz + 511) & ~511ull;
      const char type = (char)h[156];
      if (type == 'L' || type == 'x') {
        pos += 512;
        if (pos + fsz > size) {
          at_end = true;
          break;
        }
        if (type == 'L') {
          pending.assign((const char*)data + pos, (size_t)fsz);
          if (!pending.empty() && pending.back() == '\0') pending.pop_back();
        } else {
          pending = tar_pax_path(data + pos, (size_t)fsz);
        }
        pos += padded;
        continue;
      }
      if (type == '0' || type == '\0') {
        pos += 512;
        if (!pending.empty()) fp = pending;
        if (pos + fsz > size) {
          at_end = true;
          break;
        }
        path = fp;
        offsets[n] = (int64_t)pos;
        sizes[n] = (int64_t)fsz;
        pos += padded;
        found = true;
        break;
      }
      pending.clear();
      pos += 512 + padded;
    }
    if (!found) {
      if (!at_end) pos = size;
      break;
    }
    if (names && name_offs) {
      if (used + path.size() + 1 > names_cap) {
        pos = entry_pos;  // retry this entry with a fresh names buffer
        break;
      }
      memcpy(names + used, path.c_str(), path.size() + 1);
      name_offs[n] = (int64_t)used;
      used += path.size() + 1;
    }
    n++;
  }
  *n_out = n;
  *next_pos = at_end ? size : pos;
  return SPDL_HJ_OK;
}

int spdl_hj_decode_planes(spdl_hj_ctx* ctx, const uint8_t* data, size_t size, int32_t idct,
                          uint8_t* const* planes, void* stream, char* err, size_t errlen) {
  if (!ctx || !data || !planes || (idct != 0 && idct != 1)) {
    set_err(err, errlen, "invalid argument");
    return SPDL_HJ_ERR_INVALID_ARG;
  }
  DeviceGuard g(ctx->device);
  hipStream_t st = static_cast<hipStream_t>(stream);
  spdl_hj_image_info info;
  int rc = probe(data, size, &info);
  if (rc) {
    set_err(err, errlen, "Failed to decode an image. (%s)", status_str(rc));
    return rc;
  }
  spdl_hj_output o{};
  o.idct = idct;
  int64_t off = 0, sz = (int64_t)size, total = round_up(sz + 64, 256);
  Layout L;
  Slot* s = nullptr;
  hipStream_t xs;
  // (a piece hand-off that gave up: once more in one entropy workgroup)
  for (int64_t piece_bytes : {ctx->piece_bytes, (int64_t)0}) {
    L = Layout{};
    rc = build_layout(&off, &sz, &info, 1, &o, ctx->sub_bits, piece_bytes, L, nullptr, err, errlen,
                      nullptr);
    if (rc) return rc;
    rc = acquire_slot(ctx, &s, err, errlen);
    if (rc) return rc;
    HJ_HIP(s->pin_in.ensure((size_t)total));
    memcpy(s->pin_in.p, data, size);
    memset(static_cast<uint8_t*>(s->pin_in.p) + size, 0, (size_t)(total - sz));
    rc = exec_stream(ctx, *s, st, &xs, err, errlen);
    if (!rc) rc = stage_h2d(ctx, *s, (size_t)total, xs, err, errlen);
    if (rc) return rc;
    rc = run_pipeline(ctx, *s, static_cast<const uint8_t*>(s->bytes.p), (size_t)total, L, 1, &o,
                      nullptr, 0, xs, 1, nullptr, err, errlen, true);
    if (rc != SPDL_HJ_ERR_HANDOFF || piece_bytes == 0) break;
    ctx->handoff_retries++;
  }
  if (rc) return rc;
  Workspace& W = ctx->ws[s->ticket % ctx->lanes];
  st = xs;
  const ImageDesc& d = L.desc[0];
  int hmax = 1, vmax = 1;
  for (int c = 0; c < info.ncomp; c++) {
    hmax = info.h_samp[c] > hmax ? info.h_samp[c] : hmax;
    vmax = info.v_samp[c] > vmax ? info.v_samp[c] : vmax;
  }
  for (int c = 0; c < info.ncomp; c++) {
    int w = info.ncomp == 1 ? info.width : (info.width * info.h_samp[c] + hmax - 1) / hmax;
    int h = info.ncomp == 1 ? info.height : (info.height * info.v_samp[c] + vmax - 1) / vmax;
    HJ_HIP(hipMemcpy2DAsync(planes[c], (size_t)w,
                            static_cast<const uint8_t*>(W.planes.p) + d.plane_off[c],
                            (size_t)d.plane_stride[c], (size_t)w, (size_t)h,
                            hipMemcpyDeviceToHost, st));
  }
  HJ_HIP(hipStreamSynchronize(st));
  return SPDL_HJ_OK;
}

int spdl_hj_debug_entropy(spdl_hj_ctx* ctx, const uint8_t* data, size_t size, int16_t* coefs,
                          size_t coef_cap, uint8_t* clean, size_t clean_cap, int32_t* diag,
                          char* err, size_t errlen) {
  if (!ctx || !data || !diag) {
    set_err(err, errlen, "invalid argument");
    return SPDL_HJ_ERR_INVALID_ARG;
  }
  DeviceGuard g(ctx->device);
  hipStream_t st = nullptr;
  spdl_hj_image_info info;
  int rc = probe(data, size, &info);
  if (rc) {
    set_err(err, errlen, "probe failed (%s)", status_str(rc));
    return rc;
  }
  spdl_hj_output o{};
  int64_t off = 0, sz = (int64_t)size, total = round_up(sz + 64, 256);
  Layout L;
  rc = build_layout(&off, &sz, &info, 1, &o, ctx->sub_bits, ctx->piece_bytes, L, nullptr, err, errlen, nullptr);
  if (rc) return rc;
  Slot* s = nullptr;
  rc = acquire_slot(ctx, &s, err, errlen);
  if (rc) return rc;
  HJ_HIP(s->pin_in.ensure((size_t)total));
  memcpy(s->pin_in.p, data, size);
  memset(static_cast<uint8_t*>(s->pin_in.p) + size, 0, (size_t)(total - sz));
  hipStream_t xs;
  rc = exec_stream(ctx, *s, st, &xs, err, errlen);
  if (!rc) rc = stage_h2d(ctx, *s, (size_t)total, xs, err, errlen);
  if (rc) return rc;
  (void)run_pipeline(ctx, *s, static_cast<const uint8_t*>(s->bytes.p), (size_t)total, L, 1, &o,
                     nullptr, 0, xs, 1, nullptr, err, errlen, true);
  Workspace& W = ctx->ws[s->ticket % ctx->lanes];
  ImageInfo hi;
  HJ_HIP(hipMemcpy(&hi, W.info.p, sizeof(ImageInfo), hipMemcpyDeviceToHost));
  diag[0] = hi.status;
  diag[1] = hi.clean_len;
  diag[2] = hi.nseg;
  diag[3] = hi.sync_rounds;
  for (int i = 0; i < 4; i++) diag[4 + i] = (int32_t)hi.tphase[i];
  for (int i = 0; i < 4; i++) diag[8 + i] = (int32_t)hi.dbg[i];
  for (int i = 0; i < 48; i++) diag[12 + i] = hi.sdiag[i];
  // expand the coefficient lists (see BlockOut in hj_kernels.hip: entries
  // level << 16 | zig-zag index, dequantised as the IDCT does) to the dense
  // natural-order blocks the IDCT consumes
  const size_t nbk = (size_t)L.desc[0].nblocks;
  if (coefs && hi.status == SPDL_HJ_OK) {
    static const uint8_t kNatural[64] = {
        0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
        41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
        30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
    std::vector<uint2> bd(nbk);
    std::vector<uint32_t> ents(nbk * 64);
    HJ_HIP(hipMemcpy(bd.data(), W.bdesc.p, nbk * sizeof(uint2), hipMemcpyDeviceToHost));
    HJ_HIP(hipMemcpy(ents.data(), W.ents.p, nbk * 256, hipMemcpyDeviceToHost));
    std::vector<int16_t> dense(nbk * 64, 0);
    for (size_t j = 0; j < nbk; j++) {
      const int c = hi.mcu_comp[j % (size_t)hi.bpm];
      dense[j * 64] = (int16_t)(bd[j].y >> 16);
      const uint32_t cnt = bd[j].y & 0xFFFFu;
      for (uint32_t i = 0; i < cnt && bd[j].x + i < nbk * 64; i++) {
        const uint32_t e = ents[bd[j].x + i];
        const uint32_t zz = e & 63u;
        dense[j * 64 + kNatural[zz]] = (int16_t)(uint16_t)((e >> 16) * hi.qt[c][zz]);
      }
    }
    memcpy(coefs, dense.data(), 2 * (dense.size() < coef_cap ? dense.size() : coef_cap));
  }
  if (clean && hi.clean_len > 0) {
    size_t n = (size_t)hi.clean_len < clean_cap ? (size_t)hi.clean_len : clean_cap;
    HJ_HIP(hipMemcpy(clean, W.clean.p, n, hipMemcpyDeviceToHost));
  }
  return SPDL_HJ_OK;
}

int spdl_hj_nv12_to_planar_rgb(const uint8_t* src_dev, int32_t num_frames, int32_t h2,
                               int32_t width, int32_t bgr, int32_t matrix_coeff, uint8_t* dst_dev,
                               size_t dst_bytes, int device, void* stream, int32_t sync, char* err,
                               size_t errlen) {
  if (!src_dev || !dst_dev || num_frames < 0 || width <= 0 || h2 <= 0) {
    set_err(err, errlen, "invalid argument");
    return SPDL_HJ_ERR_INVALID_ARG;
  }
  if (h2 % 3 != 0) {  // reference: src/libspdl/cuda/color_conversion.cpp:45-50
    set_err(err, errlen,
            "The height of NV12 image (h*1.5) must be divisible by 3. Found: %d", (int)h2);
    return SPDL_HJ_ERR_INVALID_ARG;
  }
  const int32_t height = h2 / 3 * 2;
  if ((size_t)num_frames * 3 * height * width > dst_bytes) {
    set_err(err, errlen, "output buffer too small");
    return SPDL_HJ_ERR_INVALID_ARG;
  }
  if (matrix_coeff <= 0 || matrix_coeff > 10) matrix_coeff = 1;  // silently BT.709
  DeviceGuard g(device);
  hipStream_t st = static_cast<hipStream_t>(stream);
  HJ_HIP(launch_nv12(src_dev, dst_dev, num_frames, height, width, bgr != 0, matrix_coeff, st));
  if (sync) HJ_HIP(hipStreamSynchronize(st));
  return SPDL_HJ_OK;
}

int spdl_hj_copy(void* dst, const void* src, size_t bytes, int32_t kind, int device, void* stream,
                 int32_t pinned, char* err, size_t errlen) {
  if ((!dst || !src) && bytes) {
    set_err(err, errlen, "invalid argument");
    return SPDL_HJ_ERR_INVALID_ARG;
  }
  if (kind != 0 && kind != 1) {
    set_err(err, errlen, "invalid copy kind %d", (int)kind);
    return SPDL_HJ_ERR_INVALID_ARG;
  }
  if (!bytes) return SPDL_HJ_OK;
  DeviceGuard g(device);
  const hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost;
  if (pinned) {  // reference transfer_buffer_impl: async on the stream + sync
    hipStream_t st = static_cast<hipStream_t>(stream);
    HJ_HIP(hipMemcpyAsync(dst, src, bytes, k, st));
    HJ_HIP(hipStreamSynchronize(st));
  } else {
    HJ_HIP(hipMemcpy(dst, src, bytes, k));
  }
  return SPDL_HJ_OK;
}

int spdl_hj_set_profiling(spdl_hj_ctx* ctx, int32_t enable) {
  if (!ctx) return SPDL_HJ_ERR_INVALID_ARG;
  ctx->profiling = enable != 0;
  return SPDL_HJ_OK;
}

int spdl_hj_last_timings(spdl_hj_ctx* ctx, float* us, int32_t cap, int32_t* n_out) {
  if (!ctx || !us || !n_out) return SPDL_HJ_ERR_INVALID_ARG;
  int k = ctx->ntimings < cap ? ctx->ntimings : cap;
  for (int i = 0; i < k; i++) us[i] = ctx->timings[i];
  *n_out = k;
  return SPDL_HJ_OK;
}

const char* spdl_hj_stage_name(int32_t i) {
  return (i >= 0 && i < kStages) ? kStageNames[i] : "";
}

int spdl_hj_set_param(spdl_hj_ctx* ctx, const char* name, int64_t value) {
  if (!ctx || !name) return SPDL_HJ_ERR_INVALID_ARG;
  if (!strcmp(name, "sub_bits")) {
    if (value < 32 || value > (1 << 24) || value % 32) return SPDL_HJ_ERR_INVALID_ARG;
    ctx->sub_bits = (int)value;
    return SPDL_HJ_OK;
  }
  if (!strcmp(name, "entropy_threads")) {  // workgroup size of the Huffman kernel
    if (value != 0 && value != 128 && value != 256 && value != 512 && value != 1024)
      return SPDL_HJ_ERR_INVALID_ARG;
    ctx->entropy_threads = (int)value;
    return SPDL_HJ_OK;
  }
  if (!strcmp(name, "warmup_slots")) {  // entropy round-0 warm-up before each run
    if (value < 0 || value > 64) return SPDL_HJ_ERR_INVALID_ARG;
    ctx->warm_slots = (int)value;
    return SPDL_HJ_OK;
  }
  if (!strcmp(name, "entropy_piece_bytes")) {  // size-adaptive entropy decode; 0 = off
    if (value < 0 || (value > 0 && value < 16 * 1024)) return SPDL_HJ_ERR_INVALID_ARG;
    ctx->piece_bytes = value;
    return SPDL_HJ_OK;
  }
  if (!strcmp(name, "min_run_slots")) {  // entropy: fewest slots per run (0 = off)
    if (value < 0 || value > 64) return SPDL_HJ_ERR_INVALID_ARG;
    ctx->min_run_slots = (int)value;
    return SPDL_HJ_OK;
  }
  if (!strcmp(name, "chain_after")) {  // entropy chain rounds after this many sync rounds
    if (value < -1 || value > 15) return SPDL_HJ_ERR_INVALID_ARG;
    ctx->chain_after = (int)value;
    return SPDL_HJ_OK;
  }
  if (!strcmp(name, "parse_threads")) {
    if (value != 64 && value != 128 && value != 256) return SPDL_HJ_ERR_INVALID_ARG;
    ctx->parse_threads = (int)value;
    return SPDL_HJ_OK;
  }
  if (!strcmp(name, "entropy_prio")) {
    if (value < 0 || value > 3) return SPDL_HJ_ERR_INVALID_ARG;
    ctx->entropy_prio = (int)value;
    return SPDL_HJ_OK;
  }
  if (!strcmp(name, "sws_cols")) {  // widest swscale tile (16-256 columns; A/B knob)
    if (value < 16 || value > kSwsMaxCols) return SPDL_HJ_ERR_INVALID_ARG;
    ctx->plans.set_max_cols((int)value);
    return SPDL_HJ_OK;
  }
  if (!strcmp(name, "sws_prepass")) {  // -1 auto, 0 never, 1 always (identical outputs)
    if (value < -1 || value > 1) return SPDL_HJ_ERR_INVALID_ARG;
    ctx->plans.set_pre_mode((int)value);
    return SPDL_HJ_OK;
  }
  if (!strcmp(name, "entropy_lds_pad")) {  // bytes; > ~26 KB leaves one entropy WG per CU
    if (value < 0 || value > 64 * 1024) return SPDL_HJ_ERR_INVALID_ARG;
    ctx->entropy_lds_pad = (int)value;
    return SPDL_HJ_OK;
  }
  if (!strcmp(name, "lanes")) {  // concurrent pipelines (workspaces + streams)
    if (value < 0 || value > kMaxLanes) return SPDL_HJ_ERR_INVALID_ARG;
    // 0: automatic -- four lanes, fewer only with fewer hardware queues
    // (r04 sweep, 4-lane bench: 3 lanes 447k img/s, 4 479k, 5 431k, 8 471k)
    if (value == 0) value = std::max(1, std::min(4, ctx->hw_queues));
    // lanes beyond the hardware queues of their priority's pool would share
    // queues and serialise: clamp (spdl_hj_get_param reports the lanes in effect)
    const int lanes = std::min((int)value, std::max(1, ctx->hw_queues));
    if (!ensure_lanes(ctx, lanes)) return SPDL_HJ_ERR_HIP;
    ctx->lanes = lanes;
    return SPDL_HJ_OK;
  }
  if (!strcmp(name, "lane_priority")) {  // 1 low (own queue pool), 0 normal, -1 high
    if (value < -1 || value > 1) return SPDL_HJ_ERR_INVALID_ARG;
    if (value == ctx->lane_priority) return SPDL_HJ_OK;
    // the lanes' streams are re-created at the new priority (after their
    // work): every stream is drained first, so a failure leaves all of them
    // in place (none destroyed while lanes_ready still counts it)
    DeviceGuard g(ctx->device);
    for (Workspace& w : ctx->ws)
      if (w.stream && hipStreamSynchronize(w.stream) != hipSuccess) return SPDL_HJ_ERR_HIP;
    for (Workspace& w : ctx->ws)
      if (w.stream) {
        (void)hipStreamDestroy(w.stream);
        w.stream = nullptr;
      }
    ctx->lane_priority = (int)value;
    ctx->lanes_ready = 0;
    return ensure_lanes(ctx, std::max(1, ctx->lanes)) ? SPDL_HJ_OK : SPDL_HJ_ERR_HIP;
  }
  if (!strcmp(name, "hw_queues")) {  // the caller knows HIP initialised with another value
    if (value < 1 || value > 32) return SPDL_HJ_ERR_INVALID_ARG;
    ctx->hw_queues = (int)value;
    if (ctx->lanes > ctx->hw_queues) ctx->lanes = ctx->hw_queues;
    return SPDL_HJ_OK;
  }
  if (!strcmp(name, "output_path")) {  // equivalent output kernels (A/B and tests)
    if (value < 0 || value > 2) return SPDL_HJ_ERR_INVALID_ARG;
    ctx->output_path = (int)value;
    return SPDL_HJ_OK;
  }
  if (!strcmp(name, "ms_skip_empty")) {
    ctx->ms_skip_empty = value != 0;
    return SPDL_HJ_OK;
  }
  if (!strcmp(name, "xcd_order")) {
    if (value < 0 || value > 3) return SPDL_HJ_ERR_INVALID_ARG;
    ctx->xcd_order = (int)value;
    return SPDL_HJ_OK;
  }
  if (!strcmp(name, "lean_waits")) {
    ctx->lean_waits = value != 0;
    return SPDL_HJ_OK;
  }
  if (!strcmp(name, "profile_stages")) {  // bitmask over spdl_hj_stage_name indices
    if (value < 0 || value >= (1 << kStages)) return SPDL_HJ_ERR_INVALID_ARG;
    ctx->profile_stages = (uint32_t)value;
    return SPDL_HJ_OK;
  }
  if (!strcmp(name, "handoff_wait_us")) {  // piece hand-off wait bound (0: give up at once)
    if (value < 0 || value > 60 * 1000 * 1000) return SPDL_HJ_ERR_INVALID_ARG;
    ctx->handoff_wait_us = value;
    return SPDL_HJ_OK;
  }
  if (!strcmp(name, "host_staging")) {  // 1: kernels move descriptors / statuses; 0: DMA copies
    ctx->host_staging = value != 0;
    return SPDL_HJ_OK;
  }
#if HJ_ABLATIONS
  if (!strcmp(name, "debug_mask")) {  // timing ablations only: output is wrong
    ctx->debug_mask = (int)value;
    return SPDL_HJ_OK;
  }
#endif
  return SPDL_HJ_ERR_INVALID_ARG;
}

int spdl_hj_get_param(spdl_hj_ctx* ctx, const char* name, int64_t* value) {
  if (!ctx || !name || !value) return SPDL_HJ_ERR_INVALID_ARG;
  const int ent = ctx->entropy_threads ? ctx->entropy_threads : (ctx->lanes > 1 ? 256 : 512);
  const struct {
    const char* n;
    int64_t v;
  } tab[] = {
      {"sub_bits", ctx->sub_bits},
      {"entropy_threads", ent},
      {"warmup_slots", ctx->warm_slots >= 0 ? ctx->warm_slots : (ent <= 256 ? 6 : 12)},
      {"lanes", ctx->lanes},
      {"entropy_piece_bytes", ctx->piece_bytes},
      {"sws_prepass", ctx->plans.pre_mode()},
      {"entropy_prio", ctx->entropy_prio},
      {"min_run_slots", ctx->min_run_slots},
      {"chain_after", ctx->chain_after >= 0 ? ctx->chain_after : (ent >= 512 ? 1 : 2)},
      {"parse_threads", ctx->parse_threads},
      {"sws_cols", ctx->plans.max_cols()},
      {"hw_queues", ctx->hw_queues},
      // streams a batch holding a progressive image may use: one per lane, a
      // multiscan side stream per lane when the queues allow it, the copy stream
      {"streams", ctx->lanes * (side_streams_fit(ctx) ? 2 : 1) + 1},
      {"lane_priority", ctx->lane_priority},
      {"output_path", ctx->output_path},
      {"host_staging", ctx->host_staging},
      {"copy_threads", ctx->pool ? ctx->pool->workers() : copy_workers() + 1},
      {"device", ctx->device},
      {"handoff_wait_us", ctx->handoff_wait_us},
      {"profile_stages", ctx->profile_stages},
      {"lean_waits", ctx->lean_waits},
      {"ms_skip_empty", ctx->ms_skip_empty},
      {"xcd_order", ctx->xcd_order},
      {"handoff_retries", ctx->handoff_retries},
  };
  for (const auto& t : tab)
    if (!strcmp(name, t.n)) {
      *value = t.v;
      return SPDL_HJ_OK;
    }
  return SPDL_HJ_ERR_INVALID_ARG;
}

}  // extern "C"
