// Micro-benchmark of the single-wave (wave-uniform) decoder building blocks
// on gfx950: cycles per iteration of small loops run by ONE wave, timed with
// s_memtime.  Diagnostic only (tools/, not part of the product).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_scalar.hip -o tools/ubench_scalar
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef const uint32_t __attribute__((address_space(4)))* CW;

__device__ __forceinline__ uint32_t U(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// 0: dependent SALU chain (xor/rotate)
// 1: scalar loads, each used right away (latency chain through memory)
// 2: scalar loads prefetched one iteration ahead
// 3: v_readlane table lookup chain
// 4: ds_read + readfirstlane chain
// 5: bit reader (get(1) per iteration) over scalar-loaded words + lane-0 atomics every other bit
// 6: same as 5 without atomics
// 7: global_atomic_or from lane 0 per iteration, nothing else
__global__ void __launch_bounds__(64) ub(const uint32_t* __restrict__ data, int nwords, int iters,
                                          int mode, uint32_t* __restrict__ out,
                                          int64_t* __restrict__ cyc) {
  __shared__ uint32_t lds[1024];
  const int lane = threadIdx.x;
  for (int i = lane; i < 1024; i += 64) lds[i] = (i * 2654435761u) & 1023u;
  uint32_t tab = (lane * 40503u) & 63u;
  __syncthreads();
  CW w = (CW)(const void*)data;
  uint32_t acc = U(lane == 0 ? 1u : 0u) + 12345u;
  const int64_t t0 = (int64_t)__builtin_amdgcn_s_memtime();
  if (mode == 0) {
    for (int i = 0; i < iters; i++) {
      acc ^= acc << 7;
      acc += (acc >> 3) ^ 0x9e37u;
    }
  } else if (mode == 1) {
    uint32_t idx = 0;
    for (int i = 0; i < iters; i++) {
      const uint32_t v = w[idx];
      acc += v;
      idx = (idx + 1 + (v & 1u)) % (uint32_t)nwords;
    }
  } else if (mode == 2) {
    uint32_t idx = 0, nx = w[0];
    for (int i = 0; i < iters; i++) {
      const uint32_t v = nx;
      idx = idx + 1 < (uint32_t)nwords ? idx + 1 : 0;
      nx = w[idx];
      acc += v ^ (acc << 1);
    }
  } else if (mode == 3) {
    for (int i = 0; i < iters; i++) acc = (uint32_t)__builtin_amdgcn_readlane((int)tab, (int)(acc & 63u)) + acc;
  } else if (mode == 4) {
    for (int i = 0; i < iters; i++) acc = U(lds[acc & 1023u]) + acc;
  } else if (mode == 5 || mode == 6) {
    uint64_t buf = 0;
    int cnt = 0, pos = 0;
    for (int i = 0; i < iters; i++) {
      if (cnt < 32) {
        const uint32_t x = w[pos];
        pos = pos + 1 < nwords ? pos + 1 : 0;
        buf |= (uint64_t)U(__builtin_bswap32(x)) << (32 - cnt);
        cnt += 32;
      }
      const uint32_t bit = (uint32_t)(buf >> 63);
      buf <<= 1;
      cnt--;
      acc += bit;
      if (mode == 5 && bit && lane == 0) atomicOr(out + 64 + ((i & 1023) * 64), 1u);
    }
  } else if (mode == 8) {
    // four independent chains of the mode-0 ops (issue rate, not latency)
    uint32_t a2 = acc + 1u, a3 = acc + 2u, a4 = acc + 3u;
    for (int i = 0; i < iters; i++) {
      acc ^= acc << 7;
      a2 ^= a2 << 7;
      a3 ^= a3 << 7;
      a4 ^= a4 << 7;
      acc += (acc >> 3) ^ 0x9e37u;
      a2 += (a2 >> 3) ^ 0x9e37u;
      a3 += (a3 >> 3) ^ 0x9e37u;
      a4 += (a4 >> 3) ^ 0x9e37u;
    }
    acc ^= a2 ^ a3 ^ a4;
  } else if (mode == 9) {
    // 64-bit shifts and selects, one chain (the bit buffer's ops)
    uint64_t b = ((uint64_t)acc << 32) | 0x12345u;
    for (int i = 0; i < iters; i++) {
      const uint32_t s = (uint32_t)(b >> 59);
      b = (b << s) | (uint64_t)(s + 1u);
      b = (s & 1u) ? b ^ 0x5555ull : b;
    }
    acc += (uint32_t)b;
  } else if (mode == 10) {
    // branch taken every iteration (structurizer-style flow)
    for (int i = 0; i < iters; i++) {
      if (acc & 1u) acc = acc * 3u + 1u; else acc >>= 1;
      asm volatile("" : "+s"(acc));
    }
  } else if (mode == 7) {
    for (int i = 0; i < iters; i++)
      if (lane == 0) atomicOr(out + 64 + ((i & 1023) * 64), 1u);
  }
  const int64_t t1 = (int64_t)__builtin_amdgcn_s_memtime();
  out[lane] = acc;
  if (lane == 0) cyc[0] = t1 - t0;
}

int main() {
  const int nwords = 1 << 16, iters = 20000;
  uint32_t* h = (uint32_t*)malloc(nwords * 4);
  for (int i = 0; i < nwords; i++) h[i] = (uint32_t)(i * 2654435761u) & 0xFEFEFEFEu;
  uint32_t *d, *o;
  int64_t *c, hc;
  hipMalloc(&d, nwords * 4);
  hipMalloc(&o, (64 + 1024 * 64) * 4);
  hipMalloc(&c, 8);
  hipMemcpy(d, h, nwords * 4, hipMemcpyHostToDevice);
  const char* names[] = {"salu chain (2 dep ops)", "s_load used at once", "s_load one ahead",
                         "v_readlane chain", "ds_read+readfirstlane chain",
                         "bit reader get(1) + lane0 atomic", "bit reader get(1)",
                         "lane0 atomicOr only", "4 independent salu chains", "64-bit shift/select chain",
                         "data-dependent branch"};
  for (int m = 0; m < 11; m++) {
    for (int rep = 0; rep < 2; rep++) {
      hipLaunchKernelGGL(ub, dim3(1), dim3(64), 0, 0, d, nwords, iters, m, o, c);
      hipDeviceSynchronize();
    }
    hipMemcpy(&hc, c, 8, hipMemcpyDeviceToHost);
    printf("mode %d %-36s %8.1f cycles/iter\n", m, names[m], (double)hc / iters);
  }
  return 0;
}
