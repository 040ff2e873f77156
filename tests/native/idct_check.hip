// Device-vs-host check of the shared IDCT header (spdl_amd/csrc/hj_idct.h):
// the same source compiled for gfx950 and for the host must agree bit for bit.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../../spdl_amd/csrc/hj_idct.h"
using namespace hj;

template <int MODE>
__global__ void k_idct(const int16_t* in, uint8_t* out, int n) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  int32_t b[64], px[64];
  const uint4* src = reinterpret_cast<const uint4*>(in + (size_t)j * 64);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint4 q = src[i];
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int k = 0; k < 4; k++) {
      b[8 * i + 2 * k] = sext16(w[k]);
      b[8 * i + 2 * k + 1] = sext16(w[k] >> 16);
    }
  }
  if (MODE == 0) {
#pragma unroll
    for (int i = 0; i < 8; i++) simple_row(b + 8 * i);
#pragma unroll
    for (int i = 0; i < 8; i++) simple_col(b + i, px + i);
  } else {
    islow_block(b, px);
  }
  uint8_t* dst = out + (size_t)j * 64;
#pragma unroll
  for (int r = 0; r < 8; r++) {
    uint2 v;
    v.x = (uint32_t)px[8 * r] | ((uint32_t)px[8 * r + 1] << 8) | ((uint32_t)px[8 * r + 2] << 16) |
          ((uint32_t)px[8 * r + 3] << 24);
    v.y = (uint32_t)px[8 * r + 4] | ((uint32_t)px[8 * r + 5] << 8) |
          ((uint32_t)px[8 * r + 6] << 16) | ((uint32_t)px[8 * r + 7] << 24);
    *reinterpret_cast<uint2*>(dst + 8 * r) = v;
  }
}

int main() {
  const int n = 1 << 16;
  std::vector<int16_t> h(n * 64, 0);
  srand(3);
  for (int j = 0; j < n; j++) {
    int16_t* blk = &h[j * 64];
    blk[0] = (int16_t)(1024 + (rand() % 2048) - 1024);
    int nz = rand() % 24, range = (j % 3 == 0) ? 2000 : 600;
    for (int k = 0; k < nz; k++) blk[rand() % 64] = (int16_t)((rand() % range) - range / 2);
  }
  int16_t* din; uint8_t* dout;
  hipMalloc(&din, n * 128); hipMalloc(&dout, n * 64);
  hipMemcpy(din, h.data(), n * 128, hipMemcpyHostToDevice);
  std::vector<uint8_t> got(n * 64);
  int fails = 0;
  for (int mode = 0; mode < 2; mode++) {
    if (mode == 0) hipLaunchKernelGGL(k_idct<0>, dim3(n / 256), dim3(256), 0, 0, din, dout, n);
    else hipLaunchKernelGGL(k_idct<1>, dim3(n / 256), dim3(256), 0, 0, din, dout, n);
    hipMemcpy(got.data(), dout, n * 64, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int j = 0; j < n; j++) {
      int32_t b[64], px[64];
      for (int i = 0; i < 64; i++) b[i] = h[j * 64 + i];
      if (mode == 0) {
        for (int i = 0; i < 8; i++) simple_row(b + 8 * i);
        for (int i = 0; i < 8; i++) simple_col(b + i, px + i);
      } else {
        islow_block(b, px);
      }
      for (int i = 0; i < 64; i++)
        if ((uint8_t)px[i] != got[j * 64 + i]) {
          if (bad < 3) printf("mode %d block %d px %d: dev %d host %d\n", mode, j, i, got[j * 64 + i], px[i]);
          bad++;
        }
    }
    printf("mode %d: %d mismatching pixels of %d\n", mode, bad, n * 64);
    fails += bad;
  }
  return fails ? 1 : 0;
}
