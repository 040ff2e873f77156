/*
 * spdl_hipjpeg.h -- C-ABI of the MI355X (gfx950) JPEG decode stage.
 *
 * This is the drop-in boundary that replaces SPDL's nvJPEG/NPP stack:
 *   Python  spdl.io.decode_image_nvjpeg / load_image_batch_nvjpeg
 *           (reference src/spdl/io/_core.py:868-915, src/spdl/io/_composite.py:486-524)
 *   binding src/spdl/io/lib/cuda/decoding_nvjpeg.cpp:39-97 (nanobind, GIL released)
 *   engine  src/libspdl/cuda/nvjpeg/decoding.cpp:157-255 (decode_image_nvjpeg single/batch)
 *           src/libspdl/cuda/npp/detail/resize.cpp:36-116 (resize_npp)
 * and, for the CPU-path-compatible entry points, the FFmpeg image path behind
 *   spdl.io.load_image_batch (src/spdl/io/_composite.py:358-465).
 *
 * Plain C types only: pointers, sizes, ints.  No torch types.  Every function
 * returns 0 on success or a SPDL_HJ_ERR_* code, and writes a NUL-terminated
 * message into `err` (when non-NULL) on failure -- the Python layer turns that
 * into RuntimeError("Failed to decode an image. (...)"), matching the
 * reference's CHECK_NVJPEG behaviour (src/libspdl/cuda/nvjpeg/detail/utils.h:53-61).
 *
 * Threading: a context is used by one thread at a time (the reference keeps
 * its nvJPEG state thread_local, decoding.cpp:107-112); create one per thread.
 * Every call is GIL-free (ctypes releases the GIL).
 */
#ifndef SPDL_HIPJPEG_H
#define SPDL_HIPJPEG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPDL_HJ_ABI_VERSION 6

enum spdl_hj_status {
  SPDL_HJ_OK = 0,
  SPDL_HJ_ERR_NOT_JPEG = 1,
  SPDL_HJ_ERR_UNSUPPORTED = 2,  /* arithmetic, lossless, hierarchical, 12-bit */
  SPDL_HJ_ERR_BAD_HEADER = 3,
  SPDL_HJ_ERR_BAD_HUFFMAN = 4,
  SPDL_HJ_ERR_TRUNCATED = 5,
  SPDL_HJ_ERR_BAD_RESTART = 6,
  SPDL_HJ_ERR_BAD_GEOMETRY = 7,
  SPDL_HJ_ERR_INVALID_ARG = 8,
  SPDL_HJ_ERR_HIP = 9,
  SPDL_HJ_ERR_OOM = 10,
  /* (since ABI 6) a large restart-free file is decoded by several entropy
   * workgroups that hand run states across; a hand-off wait that polled
   * "handoff_wait_us" with nothing arriving gives up with this status.  The
   * library then re-decodes that image in one workgroup before reporting the
   * batch (spdl_hj_wait / a sync call), so callers see it only if that
   * re-decode itself fails to run. */
  SPDL_HJ_ERR_HANDOFF = 11,
};

/* output pixel formats (reference nvjpeg/detail/utils.cpp:94-110):
 * RGB/BGR planar [3,H,W]; RGB24/BGR24 interleaved [H,W,3]; YUV = raw planes. */
enum spdl_hj_pix_fmt {
  SPDL_HJ_FMT_RGB = 0,
  SPDL_HJ_FMT_BGR = 1,
  SPDL_HJ_FMT_RGB24 = 2,
  SPDL_HJ_FMT_BGR24 = 3,
};

enum spdl_hj_aspect { SPDL_HJ_ASPECT_NONE = 0, SPDL_HJ_ASPECT_DECREASE = 1, SPDL_HJ_ASPECT_INCREASE = 2 };
/* BICUBIC / BILINEAR: swscale flags of the CPU path's scale filter
 * (src/spdl/io/_preprocessing.py:214-234).  LANCZOS: Lanczos-3, the NPP
 * NPPI_INTER_LANCZOS kernel of load_image_batch_nvjpeg's resize
 * (src/libspdl/cuda/npp/detail/resize.cpp:36-116), also swscale flags=lanczos. */
enum spdl_hj_filter {
  SPDL_HJ_FILTER_BICUBIC = 0,
  SPDL_HJ_FILTER_BILINEAR = 1,
  SPDL_HJ_FILTER_LANCZOS = 2
};
/* F16 / BF16: (x/255 - mean)/std in IEEE fp32 (the reference's
 * Preprocessing.forward, examples/imagenet_classification.py:95-106), rounded
 * to nearest even into half / bfloat16. */
enum spdl_hj_dtype { SPDL_HJ_DTYPE_U8 = 0, SPDL_HJ_DTYPE_F16 = 1, SPDL_HJ_DTYPE_BF16 = 2 };
/* IDCT: FFmpeg simple_idct (the reference CPU path) or IJG islow (libjpeg). */
enum spdl_hj_idct { SPDL_HJ_IDCT_SIMPLE = 0, SPDL_HJ_IDCT_ISLOW = 1 };
/* Colour conversion / scaling: SWSCALE is the reference CPU path's libswscale
 * (one context: bicubic/bilinear/lanczos scale + yuvj -> rgb24, BT.601 full
 * range, swscale's chroma siting and fixed-point arithmetic; FilterGraphImpl,
 * src/libspdl/core/detail/ffmpeg/filter_graph.cpp:280-313).  JFIF is IJG
 * libjpeg's integer YCbCr -> RGB with nearest chroma (full resolution only). */
enum spdl_hj_csc { SPDL_HJ_CSC_SWSCALE = 0, SPDL_HJ_CSC_JFIF = 1 };

/* Output specification.  resize == 0: full resolution, every image in the
 * batch must have the same size.  Otherwise the FFmpeg filter chain SPDL
 * builds (src/spdl/io/_preprocessing.py:214-234) is applied per image:
 *   scale=w=fit_w:h=fit_h[:force_original_aspect_ratio=decrease|increase]
 *   [,pad=w=pad_w:h=pad_h:x=-1:y=-1:color=black][,crop=w=crop_w:h=crop_h]
 * fit_w/fit_h <= 0 mean "input size"; pad/crop <= 0 mean "absent". */
typedef struct spdl_hj_output {
  int32_t pix_fmt;      /* spdl_hj_pix_fmt */
  int32_t dtype;        /* spdl_hj_dtype; F16/BF16 apply (x/255 - mean)/std */
  int32_t idct;         /* spdl_hj_idct */
  int32_t resize;       /* 0 = none, 1 = apply the chain below */
  int32_t fit_w, fit_h, aspect;
  int32_t pad_w, pad_h;
  int32_t crop_w, crop_h;
  int32_t filter;       /* spdl_hj_filter */
  float mean[3], std[3];
  int32_t csc;          /* enum spdl_hj_csc, since ABI 2 */
} spdl_hj_output;

/* The frame's colour model (since ABI 4), decided at the SOF as FFmpeg's
 * mjpeg decoder picks its pix_fmt: from the Adobe APP14 transform flag seen
 * before the SOF and the component ids.
 *   GRAY    1 component                                        (gray8)
 *   YCBCR   3 components                                       (yuvj4xxp)
 *   RGB     3, Adobe transform 0 or ids 'R' 'G' 'B'; all 1x1   (gbrp)
 *   CMYK    4, all 1x1, Adobe transform 0: inverted CMYK, converted to RGB
 *           in the decoder (R = C K 257 >> 16 ...)              (gbrap)
 *   YCCK    4, Adobe transform 2: converted to YCbCr            (yuva444p)
 *   YCBCRK  4, other or no marker: YCbCr, K dropped             (yuva444p)
 * 4-component files may be sequential (interleaved or not) or progressive. */
enum spdl_hj_color {
  SPDL_HJ_COLOR_GRAY = 0,
  SPDL_HJ_COLOR_YCBCR = 1,
  SPDL_HJ_COLOR_RGB = 2,
  SPDL_HJ_COLOR_CMYK = 3,
  SPDL_HJ_COLOR_YCCK = 4,
  SPDL_HJ_COLOR_YCBCRK = 5,
};

typedef struct spdl_hj_image_info {
  int32_t width, height, ncomp;
  int32_t h_samp[4], v_samp[4];
  int32_t color;  /* enum spdl_hj_color, since ABI 4 */
  /* 1: the multi-scan path decodes the file -- progressive (SOF2), or a
   * first scan holding fewer components than the frame (since ABI 5).  A
   * batch holding such a file runs that path on a side stream beside the
   * baseline stages (spdl_hj_decode_batch_device included). */
  int32_t multiscan;
} spdl_hj_image_info;

typedef struct spdl_hj_ctx spdl_hj_ctx;

/* ABI version of the loaded library (== SPDL_HJ_ABI_VERSION). */
int spdl_hj_abi_version(void);

/* Header probe on the host: SOF fields without decoding.
 * Replaces nvjpegGetImageInfo (reference nvjpeg/decoding.cpp:114-130). */
int spdl_hj_get_image_info(const uint8_t* data, size_t size, spdl_hj_image_info* info);

/* Output geometry (width/height of the output image) for an input of w x h
 * under `out`; lets the caller allocate the output tensor. */
int spdl_hj_output_size(int32_t w, int32_t h, const spdl_hj_output* out, int32_t* out_w,
                        int32_t* out_h);

/* Create / destroy a per-thread decoder context bound to `device`.  The
 * context owns its device workspace (grown on demand) and pinned staging. */
spdl_hj_ctx* spdl_hj_create(int device, char* err, size_t errlen);
void spdl_hj_destroy(spdl_hj_ctx* ctx);

/* Decode a batch of host-resident JPEGs into caller-allocated device memory
 * `out_dev` (out_bytes long) on `stream` (a hipStream_t; NULL = legacy
 * default stream, (void*)2 = per-thread default, the reference's 0x2 sentinel
 * in src/libspdl/cuda/types.h:22-39).  The batch is packed into pinned
 * staging and copied with one hipMemcpyAsync.  Output layout per image is
 * [3,H,W] (planar) or [H,W,3] (interleaved) at offset i * per-image-size.
 * status[i] (optional, host) receives the per-image code.  With sync != 0 the
 * call returns after the stream has drained (reference default sync=true,
 * decoding.cpp:247-251) and fails if any image failed. */
int spdl_hj_decode_batch(spdl_hj_ctx* ctx, const uint8_t* const* data, const size_t* sizes,
                         int32_t n, const spdl_hj_output* out, void* out_dev, size_t out_bytes,
                         void* stream, int32_t sync, int32_t* status, char* err, size_t errlen);

/* Device-resident variant: the JPEG bytes are already in HBM, packed in
 * `dev_data` at host-known offsets (each 256-byte aligned).  `infos` are the
 * host probes of the same images (spdl_hj_get_image_info).  No H2D copy of
 * image bytes happens inside the call. */
int spdl_hj_decode_batch_device(spdl_hj_ctx* ctx, const uint8_t* dev_data, size_t dev_bytes,
                                const int64_t* offsets, const int64_t* sizes,
                                const spdl_hj_image_info* infos, int32_t n,
                                const spdl_hj_output* out, void* out_dev, size_t out_bytes,
                                void* stream, int32_t sync, int32_t* status, char* err,
                                size_t errlen);

/* ---- asynchronous submission and the pinned staging ring ----------------
 * A context owns a ring of 10 slots (pinned staging + device copy of the
 * JPEG bytes + descriptor/status staging).  Every decode call takes the next
 * slot; a call with sync == 0 returns once the batch is enqueued: the H2D copy
 * runs on the context's own copy stream and `stream` waits for it, so the host
 * can pack batch k+1 and its copy can run while batch k's kernels execute
 * (the reference copies synchronously: transfer_buffer_impl,
 * src/libspdl/cuda/transfer.cpp:37-67; transfer_tensor's pinned cache,
 * src/spdl/io/_transfer.py:82-177).  A slot is reused 10 submissions later, so
 * wait for a ticket before submitting 10 more batches or its statuses are lost. */

/* Ticket of the most recent submission on `ctx` (0 if none). */
int64_t spdl_hj_last_ticket(spdl_hj_ctx* ctx);

/* Block until the batch `ticket` has finished; per-image codes into
 * status[0..n) (optional); returns the first failure like the sync call. */
int spdl_hj_wait(spdl_hj_ctx* ctx, int64_t ticket, int32_t* status, int32_t n, char* err,
                 size_t errlen);

/* Make `stream` wait (on the device, no host block) for batch `ticket`.
 * The per-image statuses -- and the re-decode of an image whose piece
 * hand-off gave up (SPDL_HJ_ERR_HANDOFF), which rewrites its output slot --
 * come only from spdl_hj_wait: work queued on `stream` may see such an
 * image's output before spdl_hj_wait has re-decoded it. */
int spdl_hj_stream_wait(spdl_hj_ctx* ctx, int64_t ticket, void* stream, char* err,
                        size_t errlen);

/* Zero-repack ingest: take the next slot and return its pinned staging
 * (>= bytes long) so the caller can place a region of its source there
 * directly -- e.g. a run of consecutive tar members, whose payloads are
 * 512-byte aligned inside the archive (reference iter_tarfile,
 * src/spdl/io/_tar.py:33-82, yields them as zero-copy views). */
int spdl_hj_staging_acquire(spdl_hj_ctx* ctx, size_t bytes, uint8_t** host_ptr, int64_t* ticket,
                            char* err, size_t errlen);

/* Multi-threaded memcpy of host memory into an acquired slot. */
int spdl_hj_staging_fill(spdl_hj_ctx* ctx, int64_t ticket, size_t dst_off, const uint8_t* src,
                         size_t len, char* err, size_t errlen);

/* Multi-threaded pread(2) of [file_off, file_off + len) of `fd` into an
 * acquired slot (page cache -> pinned staging, no intermediate copy). */
int spdl_hj_staging_read(spdl_hj_ctx* ctx, int64_t ticket, size_t dst_off, int fd,
                         int64_t file_off, size_t len, char* err, size_t errlen);

/* Decode the images at offsets[i] (256-byte aligned), sizes[i] inside the
 * first `len` staged bytes of slot `ticket`: one hipMemcpyAsync of the whole
 * region, then the device pipeline (same output contract as
 * spdl_hj_decode_batch). */
int spdl_hj_decode_staged(spdl_hj_ctx* ctx, int64_t ticket, size_t len, const int64_t* offsets,
                          const int64_t* sizes, int32_t n, const spdl_hj_output* out,
                          void* out_dev, size_t out_bytes, void* stream, int32_t sync,
                          int32_t* status, char* err, size_t errlen);

/* Index the regular-file members of an in-memory tar archive from byte
 * `start`, at most max_entries: payload offsets/sizes, NUL-terminated names
 * concatenated into `names` (name_offs[i] indexes them; names/name_offs may
 * be NULL).  Same member walk as the reference's InMemoryTarParserImpl
 * (src/spdl/io/lib/archive/tar_iterator.cpp:125-195: ustar magic + checksum,
 * GNU 'L' long names, pax 'x' path records, empty name = end).  *next_pos is
 * where to resume (== size at the end of the archive). */
int spdl_hj_tar_index(const uint8_t* data, size_t size, size_t start, int32_t max_entries,
                      int64_t* offsets, int64_t* sizes, int64_t* name_offs, char* names,
                      size_t names_cap, int32_t* n_out, size_t* next_pos);

/* Raw decoded planes (parity surface, the reference's load_image with
 * filter_desc=None -> yuvj4xxp planes, src/spdl/io/_composite.py:254-295):
 * plane c of image 0 copied to host buffer planes[c] (comp_w x comp_h bytes,
 * tightly packed).  Single image. */
int spdl_hj_decode_planes(spdl_hj_ctx* ctx, const uint8_t* data, size_t size, int32_t idct,
                          uint8_t* const* planes, void* stream, char* err, size_t errlen);

/* Debug/parity surface: run parse + destuff + entropy decode of one image
 * and copy back the dequantised coefficients (nblocks x 64 int16, natural
 * order, MCU order, DC carries the FFmpeg +1024 bias), the destuffed scan
 * bytes, and diagnostics diag[0..3] = {status, clean_len, nseg, sync_rounds},
 * diag[4..7] = entropy phase durations (wall_clock64 ticks, 100 MHz) for
 * round 0, sync rounds, prefix scan, write pass; diag[8..11] debug counters
 * (round-0 symbols, wave iterations, shader clocks, realtime ticks);
 * diag[12 + 3 s .. 14 + 3 s] multi-scan images, scan s < 16: start and end
 * (realtime ticks from the decode start) and Huffman symbols; diag must hold
 * 60 ints. */
int spdl_hj_debug_entropy(spdl_hj_ctx* ctx, const uint8_t* data, size_t size, int16_t* coefs,
                          size_t coef_cap, uint8_t* clean, size_t clean_cap, int32_t* diag,
                          char* err, size_t errlen);

/* Batched NV12 -> planar RGB (bgr == 0) or BGR: src_dev is
 * [num_frames, h2 = 1.5 H, width] u8 in device memory (pitch = width), dst_dev
 * [num_frames, 3, H, width] u8.  matrix_coeff selects the matrix (1 BT.709
 * default, 4 FCC, 5 BT.470, 6 BT.601, 7 SMPTE240M, 8 YCgCo, 9 BT.2020,
 * 10 BT.2020C; other values mean 1).  Replaces nv12_to_planar_rgb/bgr
 * (reference src/libspdl/cuda/color_conversion.cpp:27-95,
 * detail/color_conversion.cu:90-138); like it, quads with x + 1 >= width are
 * not written.  Needs no context (stateless). */
int spdl_hj_nv12_to_planar_rgb(const uint8_t* src_dev, int32_t num_frames, int32_t h2,
                               int32_t width, int32_t bgr, int32_t matrix_coeff, uint8_t* dst_dev,
                               size_t dst_bytes, int device, void* stream, int32_t sync, char* err,
                               size_t errlen);

/* Host <-> device copy of `bytes` (kind 0: host -> device, 1: device ->
 * host).  pinned != 0: hipMemcpyAsync on `stream`, then the stream is
 * synchronised; otherwise a synchronous hipMemcpy.  Replaces
 * transfer_buffer_impl / transfer_buffer (reference
 * src/libspdl/cuda/transfer.cpp:37-105). */
int spdl_hj_copy(void* dst, const void* src, size_t bytes, int32_t kind, int device, void* stream,
                 int32_t pinned, char* err, size_t errlen);

/* Per-stage timing of the last batch, in microseconds, measured with HIP
 * events on the decode stream (filled only when enabled; -1 for a stage
 * outside "profile_stages").  The "idct" stage
 * includes the multi-scan launch (or the wait for its side stream). */
int spdl_hj_set_profiling(spdl_hj_ctx* ctx, int32_t enable);
int spdl_hj_last_timings(spdl_hj_ctx* ctx, float* us, int32_t cap, int32_t* n_out);
/* Names of the timed stages in the order spdl_hj_last_timings reports them. */
const char* spdl_hj_stage_name(int32_t i);

/* Tuning knobs: "sub_bits" (slot size of the parallel Huffman decode,
 * default 384), "entropy_threads" (256/512/1024; default 512 with one lane,
 * 256 with more), "warmup_slots" (0-64: slots a Huffman run decodes from a
 * guessed state before its own first slot; default 6 with 256 threads, 12
 * with more), "lanes" (1-8 concurrent pipelines, 0 = automatic: 4, or the
 * hardware queues when fewer; with N > 1, successive
 * batches rotate over N device workspaces and run on the context's own N
 * streams, each ordered after the caller's stream at submission; completion
 * is then observed through the ticket -- spdl_hj_wait / spdl_hj_stream_wait
 * -- not by the caller's stream; each lane wants a hardware queue of its own,
 * so the value is clamped to "hw_queues"; a lane's stream is created when
 * first enabled), "lane_priority" (stream priority of the lanes: 1 = low,
 * the default, 0 = normal, -1 = high; HIP keeps up to "hw_queues" hardware
 * queues per priority, so low-priority lanes get queues of their own beside
 * the normal-priority null / torch streams; changing it re-creates the lane
 * streams after their work), "hw_queues" (hardware queues per priority pool:
 * read from GPU_MAX_HW_QUEUES at spdl_hj_create, default 4; set it when HIP
 * initialised with another value), "output_path" (0 = by
 * batch, 1 = the generic swscale kernel, 2 = separate IDCT + unscaled
 * converter at full resolution: byte-identical outputs, for A/B and tests),
 * "entropy_piece_bytes" (size-adaptive Huffman decode: a file larger than
 * this is decoded by ceil(size / value) workgroups, at most 64; default
 * 131072, 0 = one workgroup per image; since ABI 5 round 5), "sws_prepass"
 * (-1 = automatic: the horizontal scaling pass of a downscale by >= 4x or
 * with a > 64-tap filter runs once per source row in its own kernel; 0 =
 * never, 1 = always; byte-identical outputs), "handoff_wait_us" (ABI 6: the
 * bound of a piece hand-off wait, in microseconds of polling with no awaited
 * record arriving -- time while the waves are switched out does not count;
 * default 2000000; 0 gives up at once, which only tests use: every image
 * whose pieces would have waited is re-decoded in one workgroup).
 * "chain_after" (ABI 6: entropy sync rounds after which runs still out of
 * step with their left neighbour are re-decoded chain by chain by whole
 * waves; default -1 = 1 with 512+ entropy threads, 2 with fewer; 0 =
 * never; byte-identical outputs), "min_run_slots"
 * (ABI 6: the fewest slots an entropy run decodes; default 0 = one run per
 * thread; byte-identical outputs),
 * "profile_stages" (ABI 6: bitmask of the stages, by spdl_hj_stage_name
 * index, whose HIP events are recorded while profiling; default all; stages
 * outside it report -1), "lean_waits" (ABI 6: 1, the default, skips the
 * cross-stream event waits stream order already implies -- a workspace's
 * previous batch on the same stream, a caller stream with nothing pending;
 * 0 = always wait), "xcd_order" (ABI 6: XCD-aware tile order, bit 0 the
 * swscale kernel, bit 1 the IDCT kernel; default 1; byte-identical outputs).
 * A/B knobs, byte-identical outputs: "entropy_prio" (0-3, s_setprio of the
 * entropy waves; default 0), "parse_threads" (64/128/256; default 64),
 * "sws_cols" (16-256 output columns per swscale workgroup; default 256),
 * "entropy_lds_pad" (extra LDS bytes per entropy workgroup; default 0),
 * "ms_skip_empty" (1: skip the multi-scan launch of a batch known to hold
 * no multi-scan image; default 0), "host_staging" (1, the default: kernels
 * move descriptors / statuses through mapped pinned memory; 0: DMA copies).
 * Read-only (spdl_hj_get_param): "handoff_retries", images re-decoded after a
 * hand-off gave up, since the context was created; "streams", the HIP
 * streams a batch holding a progressive image may use (one per lane, a
 * multi-scan side stream per lane when the hardware queues allow, the copy
 * stream).
 * Builds with -DHJ_ABLATIONS=1 also take "debug_mask" (timing ablations that
 * skip kernel phases; outputs wrong); release builds reject it. */
int spdl_hj_set_param(spdl_hj_ctx* ctx, const char* name, int64_t value);

/* Value in effect of a knob above (ABI 3), or of "copy_threads" (host
 * threads packing pinned staging) / "device". */
int spdl_hj_get_param(spdl_hj_ctx* ctx, const char* name, int64_t* value);

#ifdef __cplusplus
}
#endif
#endif
