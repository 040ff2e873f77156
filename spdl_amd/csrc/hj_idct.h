// hj_idct.h -- 8x8 IDCTs of idct_kernel (FFmpeg simple_idct 8-bit and IJG
// islow), bit-exact to the oracle's (tests/test_gpu_parity.py planes tests).
// HJ_HD marks functions that also compile for the host.
#pragma once
#include <stdint.h>

#ifndef HJ_HD
#define HJ_HD __host__ __device__
#endif

namespace hj {

#ifndef HJ_DC_BIAS_DEFINED
#define HJ_DC_BIAS_DEFINED
#endif

constexpr int kW1 = 22725, kW2 = 21407, kW3 = 19266, kW4 = 16383, kW5 = 12873, kW6 = 8867,
              kW7 = 4520;

HJ_HD inline uint8_t clip_u8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

// Clamp to u8 and hide the result from instruction selection.  On gfx950,
// hipcc (ROCm 7.2) fuses pairs of clip_u8(x >> k) feeding a byte-pack into
// v_ashr_pk_u8_i32 and then ORs the other bytes of the word into its result
// as if bits [31:16] were zero; measured on MI355X that corrupts bytes 2..3
// of the packed word (tests/native/idct_check.hip reproduces it).  The empty
// asm makes the clamped value opaque, so no fused pack is formed.
HJ_HD inline int32_t clip_u8_opaque(int v) {
  int32_t r = v < 0 ? 0 : (v > 255 ? 255 : v);
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(r));
#endif
  return r;
}

// FFmpeg simple_idct 8-bit (see oracle/jpeg_oracle.c simple_row / simple_col_put).
// Straight-line form: values live in int32 registers, the row results are
// truncated to int16 exactly like FFmpeg's in-place int16 rows, the sparse
// "if (row[k])" tests are dropped (they only skip additions of zero) and the
// DC-only row shortcut (row[0] << 3, as int16) is a select.
HJ_HD inline int32_t sext16(uint32_t v) { return (int32_t)(int16_t)(uint16_t)v; }

// NC = 4: the caller knows r[4..7] are zero (the terms they feed vanish;
// same results).
template <int NC = 8>
HJ_HD inline void simple_row(int32_t* r) {
  const uint32_t u0 = (uint32_t)r[0], u1 = (uint32_t)r[1], u2 = (uint32_t)r[2],
                 u3 = (uint32_t)r[3], u4 = NC > 4 ? (uint32_t)r[4] : 0u,
                 u5 = NC > 4 ? (uint32_t)r[5] : 0u, u6 = NC > 4 ? (uint32_t)r[6] : 0u,
                 u7 = NC > 4 ? (uint32_t)r[7] : 0u;
  const bool dc_only = !(u1 | u2 | u3 | u4 | u5 | u6 | u7);
  uint32_t a0 = (uint32_t)kW4 * u0 + (1u << 10);
  uint32_t a1 = a0, a2 = a0, a3 = a0;
  a0 += (uint32_t)kW2 * u2;
  a1 += (uint32_t)kW6 * u2;
  a2 -= (uint32_t)kW6 * u2;
  a3 -= (uint32_t)kW2 * u2;
  uint32_t b0 = (uint32_t)kW1 * u1 + (uint32_t)kW3 * u3;
  uint32_t b1 = (uint32_t)kW3 * u1 - (uint32_t)kW7 * u3;
  uint32_t b2 = (uint32_t)kW5 * u1 - (uint32_t)kW1 * u3;
  uint32_t b3 = (uint32_t)kW7 * u1 - (uint32_t)kW5 * u3;
  a0 += (uint32_t)kW4 * u4 + (uint32_t)kW6 * u6;
  a1 += (uint32_t)(-kW4) * u4 - (uint32_t)kW2 * u6;
  a2 += (uint32_t)(-kW4) * u4 + (uint32_t)kW2 * u6;
  a3 += (uint32_t)kW4 * u4 - (uint32_t)kW6 * u6;
  b0 += (uint32_t)kW5 * u5 + (uint32_t)kW7 * u7;
  b1 += (uint32_t)(-kW1) * u5 - (uint32_t)kW5 * u7;
  b2 += (uint32_t)kW7 * u5 + (uint32_t)kW3 * u7;
  b3 += (uint32_t)kW3 * u5 - (uint32_t)kW1 * u7;
  const int32_t dc = sext16(u0 << 3);
  r[0] = dc_only ? dc : sext16((uint32_t)((int32_t)(a0 + b0) >> 11));
  r[7] = dc_only ? dc : sext16((uint32_t)((int32_t)(a0 - b0) >> 11));
  r[1] = dc_only ? dc : sext16((uint32_t)((int32_t)(a1 + b1) >> 11));
  r[6] = dc_only ? dc : sext16((uint32_t)((int32_t)(a1 - b1) >> 11));
  r[2] = dc_only ? dc : sext16((uint32_t)((int32_t)(a2 + b2) >> 11));
  r[5] = dc_only ? dc : sext16((uint32_t)((int32_t)(a2 - b2) >> 11));
  r[3] = dc_only ? dc : sext16((uint32_t)((int32_t)(a3 + b3) >> 11));
  r[4] = dc_only ? dc : sext16((uint32_t)((int32_t)(a3 - b3) >> 11));
}

// column k of the row-pass output: c[8*j], j = 0..7; writes 8 pixels o[8*j].
// NR = 4: the caller knows rows 4..7 are zero.
template <int NR = 8>
HJ_HD inline void simple_col(const int32_t* c, int32_t* o) {
  const uint32_t u1 = (uint32_t)c[8], u2 = (uint32_t)c[16], u3 = (uint32_t)c[24],
                 u4 = NR > 4 ? (uint32_t)c[32] : 0u, u5 = NR > 4 ? (uint32_t)c[40] : 0u,
                 u6 = NR > 4 ? (uint32_t)c[48] : 0u, u7 = NR > 4 ? (uint32_t)c[56] : 0u;
  uint32_t a0 = (uint32_t)kW4 * (uint32_t)(c[0] + ((1 << 19) / kW4));
  uint32_t a1 = a0, a2 = a0, a3 = a0;
  a0 += (uint32_t)kW2 * u2;
  a1 += (uint32_t)kW6 * u2;
  a2 -= (uint32_t)kW6 * u2;
  a3 -= (uint32_t)kW2 * u2;
  uint32_t b0 = (uint32_t)kW1 * u1 + (uint32_t)kW3 * u3;
  uint32_t b1 = (uint32_t)kW3 * u1 - (uint32_t)kW7 * u3;
  uint32_t b2 = (uint32_t)kW5 * u1 - (uint32_t)kW1 * u3;
  uint32_t b3 = (uint32_t)kW7 * u1 - (uint32_t)kW5 * u3;
  a0 += (uint32_t)kW4 * u4;
  a1 -= (uint32_t)kW4 * u4;
  a2 -= (uint32_t)kW4 * u4;
  a3 += (uint32_t)kW4 * u4;
  b0 += (uint32_t)kW5 * u5;
  b1 -= (uint32_t)kW1 * u5;
  b2 += (uint32_t)kW7 * u5;
  b3 += (uint32_t)kW3 * u5;
  a0 += (uint32_t)kW6 * u6;
  a1 -= (uint32_t)kW2 * u6;
  a2 += (uint32_t)kW2 * u6;
  a3 -= (uint32_t)kW6 * u6;
  b0 += (uint32_t)kW7 * u7;
  b1 -= (uint32_t)kW5 * u7;
  b2 += (uint32_t)kW3 * u7;
  b3 -= (uint32_t)kW1 * u7;
  o[0] = clip_u8_opaque((int32_t)(a0 + b0) >> 20);
  o[8] = clip_u8_opaque((int32_t)(a1 + b1) >> 20);
  o[16] = clip_u8_opaque((int32_t)(a2 + b2) >> 20);
  o[24] = clip_u8_opaque((int32_t)(a3 + b3) >> 20);
  o[32] = clip_u8_opaque((int32_t)(a3 - b3) >> 20);
  o[40] = clip_u8_opaque((int32_t)(a2 - b2) >> 20);
  o[48] = clip_u8_opaque((int32_t)(a1 - b1) >> 20);
  o[56] = clip_u8_opaque((int32_t)(a0 - b0) >> 20);
}

// IJG islow (see oracle/jpeg_oracle.c jo_idct_islow)
constexpr int F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373,
              F1175 = 9633, F1501 = 12299, F1847 = 15137, F1961 = 16069, F2053 = 16819,
              F2562 = 20995, F3072 = 25172;

HJ_HD inline uint8_t islow_limit(int32_t x) {
  const int v = (int)(x & 1023) - 384;
  return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

HJ_HD inline void islow_block(int32_t* in, int32_t* out) {
  int32_t ws[64];
  in[0] = sext16((uint32_t)(in[0] - 1024));
#pragma unroll
  for (int c = 0; c < 8; c++) {
    const int32_t* p = in + c;
    if (!(p[8] | p[16] | p[24] | p[32] | p[40] | p[48] | p[56])) {
      const int32_t dc = (int32_t)p[0] * 4;
#pragma unroll
      for (int r = 0; r < 8; r++) ws[r * 8 + c] = dc;
      continue;
    }
    int32_t z1, z2, z3, t0, t1, t2, t3, t10, t11, t12, t13;
    z2 = (int32_t)p[0] * 8192 + (1 << 10);
    z3 = (int32_t)p[32] * 8192;
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
    z2 = z2 * -F1961 + z1;
    z3 = z3 * -F0390 + z1;
    z1 = (t0 + t3) * -F0899;
    t0 = t0 * F0298 + z1 + z2;
    t3 = t3 * F1501 + z1 + z3;
    z1 = (t1 + t2) * -F2562;
    t1 = t1 * F2053 + z1 + z3;
    t2 = t2 * F3072 + z1 + z2;
    ws[0 * 8 + c] = (t10 + t3) >> 11;
    ws[7 * 8 + c] = (t10 - t3) >> 11;
    ws[1 * 8 + c] = (t11 + t2) >> 11;
    ws[6 * 8 + c] = (t11 - t2) >> 11;
    ws[2 * 8 + c] = (t12 + t1) >> 11;
    ws[5 * 8 + c] = (t12 - t1) >> 11;
    ws[3 * 8 + c] = (t13 + t0) >> 11;
    ws[4 * 8 + c] = (t13 - t0) >> 11;
  }
#pragma unroll
  for (int r = 0; r < 8; r++) {
    const int32_t* w = ws + r * 8;
    int32_t* o = out + r * 8;
    int32_t z1, z2, z3, t0, t1, t2, t3, t10, t11, t12, t13;
    z2 = w[0] + ((512 << 5) + (1 << 4));
    if (!(w[1] | w[2] | w[3] | w[4] | w[5] | w[6] | w[7])) {
      const int32_t v = islow_limit(z2 >> 5);
#pragma unroll
      for (int i = 0; i < 8; i++) o[i] = v;
      continue;
    }
    z3 = w[4];
    t0 = (z2 + z3) * 8192;
    t1 = (z2 - z3) * 8192;
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
    z2 = z2 * -F1961 + z1;
    z3 = z3 * -F0390 + z1;
    z1 = (t0 + t3) * -F0899;
    t0 = t0 * F0298 + z1 + z2;
    t3 = t3 * F1501 + z1 + z3;
    z1 = (t1 + t2) * -F2562;
    t1 = t1 * F2053 + z1 + z3;
    t2 = t2 * F3072 + z1 + z2;
    o[0] = islow_limit((t10 + t3) >> 18);
    o[7] = islow_limit((t10 - t3) >> 18);
    o[1] = islow_limit((t11 + t2) >> 18);
    o[6] = islow_limit((t11 - t2) >> 18);
    o[2] = islow_limit((t12 + t1) >> 18);
    o[5] = islow_limit((t12 - t1) >> 18);
    o[3] = islow_limit((t13 + t0) >> 18);
    o[4] = islow_limit((t13 - t0) >> 18);
  }
}


}  // namespace hj
