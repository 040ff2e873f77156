// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// patterns of this project's kernels (MI355X_MICROARCH.md §HBM: the x2
// FETCH correction is calibrated only for wide coalesced streaming reads;
// "calibrate on a known byte count in your own access pattern").
//
// Every kernel touches each byte of a fresh 1 GiB buffer exactly once (far
// past the 256 MiB Infinity Cache), so the true fabric traffic per dispatch
// is the byte count printed; the counters' per-dispatch values divided by
// it give each pattern's correction factor.
//
//   stream_read   16 B per lane, consecutive lanes consecutive (reference)
//   window_read   entropy_kernel's bit-reader restage: each lane reads 32 B
//                 (two dword-aligned 16-B loads) at its own position, lanes
//                 ~3.4 KB apart, advancing through their own streams
//   list_read     idct_kernel's coefficient lists: each lane reads a run of
//                 16-B groups of its own, lanes' runs adjacent
//   stream_write  16 B per lane coalesced (reference)
//   append_write  entropy_kernel's list stores: each lane appends 16-B
//                 groups to its own region, lanes ~3.4 KB apart
//   rows_write    idct_kernel's plane stores: 8 B per lane per row, a
//                 lane's 8 rows one plane stride apart
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip
// run:   rocprofv3 --kernel-trace --pmc FETCH_SIZE -- ./tools/fetch_calib   (and WRITE_SIZE)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr size_t kBytes = size_t(1) << 30;
constexpr int kThreads = 256;

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__global__ void stream_read(const uint4* __restrict__ p, size_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 q = p[i];
    acc ^= q.x ^ q.y ^ q.z ^ q.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// lane l owns the stream [l * span, (l + 1) * span) bytes and reads it 32 B
// at a time from dword-aligned (not 16-B aligned) positions, as win_stage
constexpr size_t kSpan = 3392;  // ~ one entropy run's bytes at 256 runs per 108 KB image
__global__ void window_read(const uint8_t* __restrict__ p, size_t lanes, uint32_t* sink) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4), aligned(4)));
  const size_t l = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (l >= lanes) return;
  const uint8_t* base = p + l * kSpan;
  uint32_t acc = 0;
  for (size_t off = 4; off + 32 <= kSpan; off += 32) {
    const u32x4* q = reinterpret_cast<const u32x4*>(base + off);
    const u32x4 a = q[0], b = q[1];
    acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// lane l reads its own run of 16-B groups (a block's list: 1..16 groups)
__global__ void list_read(const uint4* __restrict__ p, size_t lanes, uint32_t* sink) {
  const size_t l = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (l >= lanes) return;
  const uint4* q = p + l * 8;  // 8 groups = 32 entries per list
  uint32_t acc = 0;
  for (int i = 0; i < 8; i++) acc ^= q[i].x ^ q[i].y ^ q[i].z ^ q[i].w;
  if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void stream_write(uint4* __restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

__global__ void append_write(uint8_t* __restrict__ p, size_t lanes) {
  const size_t l = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (l >= lanes) return;
  uint4* q = reinterpret_cast<uint4*>(p + l * kSpan);
  for (size_t i = 0; i < kSpan / 16; i++) q[i] = make_uint4((uint32_t)i, (uint32_t)l, 2u, 3u);
}

// lanes = blocks of an 8-row band: lane l writes 8 B at row r, column l
__global__ void rows_write(uint8_t* __restrict__ p, size_t width, size_t bands) {
  const size_t l = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const size_t cols = width / 8;
  if (l >= cols * bands) return;
  const size_t band = l / cols, col = l % cols;
  uint8_t* dst = p + band * 8 * width + col * 8;
  for (int r = 0; r < 8; r++)
    *reinterpret_cast<uint2*>(dst + r * width) = make_uint2((uint32_t)l, (uint32_t)r);
}

int main() {
  uint8_t* buf;
  uint32_t* sink;
  CHECK(hipMalloc(&buf, kBytes));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMemset(buf, 1, kBytes));
  CHECK(hipDeviceSynchronize());
  const int grid = 8192;
  // read patterns over the whole buffer
  hipLaunchKernelGGL(stream_read, dim3(grid), dim3(kThreads), 0, 0,
                     reinterpret_cast<const uint4*>(buf), kBytes / 16, sink);
  CHECK(hipDeviceSynchronize());
  printf("stream_read %zu bytes\n", kBytes);
  {
    const size_t lanes = kBytes / kSpan;
    hipLaunchKernelGGL(window_read, dim3((lanes + kThreads - 1) / kThreads), dim3(kThreads), 0, 0,
                       buf, lanes, sink);
    CHECK(hipDeviceSynchronize());
    // bytes [4, 4 + 32 * floor((span - 4) / 32)) of each lane's stream
    printf("window_read %zu bytes\n", lanes * ((kSpan - 4) / 32 * 32));
  }
  {
    const size_t lanes = kBytes / 128;
    hipLaunchKernelGGL(list_read, dim3((lanes + kThreads - 1) / kThreads), dim3(kThreads), 0, 0,
                       reinterpret_cast<const uint4*>(buf), lanes, sink);
    CHECK(hipDeviceSynchronize());
    printf("list_read %zu bytes\n", lanes * 128);
  }
  hipLaunchKernelGGL(stream_write, dim3(grid), dim3(kThreads), 0, 0, reinterpret_cast<uint4*>(buf),
                     kBytes / 16);
  CHECK(hipDeviceSynchronize());
  printf("stream_write %zu bytes\n", kBytes);
  {
    const size_t lanes = kBytes / kSpan;
    hipLaunchKernelGGL(append_write, dim3((lanes + kThreads - 1) / kThreads), dim3(kThreads), 0, 0,
                       buf, lanes);
    CHECK(hipDeviceSynchronize());
    printf("append_write %zu bytes\n", lanes * (kSpan / 16 * 16));
  }
  {
    const size_t width = 640, bands = kBytes / (8 * width);
    const size_t lanes = bands * (width / 8);
    hipLaunchKernelGGL(rows_write, dim3((lanes + kThreads - 1) / kThreads), dim3(kThreads), 0, 0, buf,
                       width, bands);
    CHECK(hipDeviceSynchronize());
    printf("rows_write %zu bytes\n", bands * 8 * width);
  }
  CHECK(hipFree(buf));
  CHECK(hipFree(sink));
  return 0;
}
