// Packed-fp32 complex arithmetic and the DFT building blocks of the MFCC
// kernel's 512-point real FFT (gfx950).
//
// A complex value is one 64-bit VGPR pair (v2f = {re, im}); every complex
// add / sub / multiply is one or two v_pk_* instructions (two fp32 lanes per
// instruction, the only way to reach the chip's 157 TF fp32 rate).  The
// multiplications by -i, the conjugations and the swizzles that CDNA4's VOP3P
// op_sel / neg modifiers express for free are written as inline asm: the
// compiler otherwise materialises them with v_xor / v_mov.
#pragma once

#include <hip/hip_runtime.h>

namespace vad {

typedef float v2f __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));

constexpr float kC8 = 0.70710678118654752440f;   // cos(pi/4)
constexpr float kC16 = 0.92387953251128675613f;  // cos(pi/8)
constexpr float kS16 = 0.38268343236508977173f;  // sin(pi/8)

namespace pk {

// a * w
__device__ __forceinline__ v2f cmul(v2f a, v2f w) {
  v2f t, d;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(a), "v"(w));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
      : "=v"(d) : "v"(a), "v"(w), "v"(t));
  return d;
}
// a + (-i) b = (a.x + b.y, a.y - b.x)
__device__ __forceinline__ v2f add_mi(v2f a, v2f b) {
  v2f d;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
// a - (-i) b = (a.x - b.y, a.y + b.x)
__device__ __forceinline__ v2f sub_mi(v2f a, v2f b) {
  v2f d;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
// a + conj(b) = (a.x + b.x, a.y - b.y)
__device__ __forceinline__ v2f add_conj(v2f a, v2f b) {
  v2f d;
  asm("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
// a - conj(b) = (a.x - b.x, a.y + b.y)
__device__ __forceinline__ v2f sub_conj(v2f a, v2f b) {
  v2f d;
  asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1]" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
// (s.x + t.y, s.x - t.y)
__device__ __forceinline__ v2f split_u(v2f s, v2f t) {
  v2f d;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[0,1] neg_hi:[0,1]" : "=v"(d) : "v"(s), "v"(t));
  return d;
}
// (s.y - t.x, -s.y - t.x)
__device__ __forceinline__ v2f split_v(v2f s, v2f t) {
  v2f d;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[1,1]"
      : "=v"(d) : "v"(s), "v"(t));
  return d;
}
// a * (c - i s) = c a + s (a.y, -a.x), c and s compile-time constants
template <int CI, int SI>
__device__ __forceinline__ v2f mul_cs(v2f a) {
  constexpr float c = __builtin_bit_cast(float, CI), s = __builtin_bit_cast(float, SI);
  const v2f t = a * c;
  const v2f ss = {s, s};
  v2f d;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,1,1] neg_hi:[1,0,0]"
      : "=v"(d) : "v"(a), "s"(ss), "v"(t));
  return d;
}
constexpr int kC16i = __builtin_bit_cast(int, kC16);
constexpr int kS16i = __builtin_bit_cast(int, kS16);
constexpr int kmC16i = __builtin_bit_cast(int, -kC16);
constexpr int kmS16i = __builtin_bit_cast(int, -kS16);

__device__ __forceinline__ v2f w16_1(v2f a) { return mul_cs<kC16i, kS16i>(a); }    // W16^1
__device__ __forceinline__ v2f w16_3(v2f a) { return mul_cs<kS16i, kC16i>(a); }    // W16^3
__device__ __forceinline__ v2f w16_5(v2f a) { return mul_cs<kmS16i, kC16i>(a); }   // W16^5
__device__ __forceinline__ v2f w16_7(v2f a) { return mul_cs<kmC16i, kS16i>(a); }   // W16^7
__device__ __forceinline__ v2f w8_1(v2f a) { return add_mi(a, a) * kC8; }          // W8^1 = W16^2

// forward DFT4 (W4 = -i); y2, y3 given as x2 = (-i) y2, x3 = (-i) y3 when MI23;
// Z3: x3 is a known zero (the zero padding of the frame), so x1 +- x3 = x1
// (the compiler may not fold x1 + 0: -0 + 0 = +0)
template <bool MI23 = false, bool Z3 = false>
__device__ __forceinline__ void dft4(v2f& x0, v2f& x1, v2f& x2, v2f& x3) {
  v2f t0, t1, t2, t3;
  if constexpr (MI23) {
    t0 = add_mi(x0, x2); t1 = sub_mi(x0, x2);
    t2 = add_mi(x1, x3); t3 = sub_mi(x1, x3);
  } else if constexpr (Z3) {
    t0 = x0 + x2; t1 = x0 - x2;
    t2 = x1; t3 = x1;
  } else {
    t0 = x0 + x2; t1 = x0 - x2;
    t2 = x1 + x3; t3 = x1 - x3;
  }
  x0 = t0 + t2;
  x2 = t0 - t2;
  x1 = add_mi(t1, t3);
  x3 = sub_mi(t1, t3);
}

// forward DFT8, natural order; MI46: x4, x6 are given divided by -i
template <bool MI46 = false>
__device__ __forceinline__ void dft8(v2f (&x)[8]) {
  v2f e0 = x[0], e1 = x[2], e2 = x[4], e3 = x[6];
  v2f o0 = x[1], o1 = x[3], o2 = x[5], o3 = x[7];
  dft4<MI46>(e0, e1, e2, e3);
  dft4(o0, o1, o2, o3);
  const v2f w1 = w8_1(o1);   // W8^1 o1
  const v2f w3 = w8_1(o3);   // W8^3 o3 = (-i) w3
  x[0] = e0 + o0; x[4] = e0 - o0;
  x[1] = e1 + w1; x[5] = e1 - w1;
  x[2] = add_mi(e2, o2); x[6] = sub_mi(e2, o2);
  x[3] = add_mi(e3, w3); x[7] = sub_mi(e3, w3);
}

// forward DFT16 in place, natural order; x[n >= NZ] are known zeros.
// 4x4 Cooley-Tukey: n = 4a + b, k = c + 4d.
template <int NZ>
__device__ __forceinline__ void dft16(v2f (&x)[16]) {
#pragma unroll
  for (int n = NZ; n < 16; ++n) x[n] = (v2f){0.f, 0.f};
  v2f v[4][4];
  static_assert(NZ > 12, "the first-stage DFT4s assume x[0..12] may be non-zero");
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    v2f a0 = x[b], a1 = x[4 + b], a2 = x[8 + b], a3 = x[12 + b];
    if (12 + b >= NZ) dft4<false, true>(a0, a1, a2, a3);
    else dft4(a0, a1, a2, a3);
    v[b][0] = a0; v[b][1] = a1; v[b][2] = a2; v[b][3] = a3;
  }
  // c = 0: no twiddles
  { v2f b0 = v[0][0], b1 = v[1][0], b2 = v[2][0], b3 = v[3][0];
    dft4(b0, b1, b2, b3); x[0] = b0; x[4] = b1; x[8] = b2; x[12] = b3; }
  // c = 1: W16^1, W16^2, W16^3
  { v2f b0 = v[0][1], b1 = w16_1(v[1][1]), b2 = w8_1(v[2][1]), b3 = w16_3(v[3][1]);
    dft4(b0, b1, b2, b3); x[1] = b0; x[5] = b1; x[9] = b2; x[13] = b3; }
  // c = 2: W16^2, W16^4 = -i, W16^6 = (-i) W16^2 -> fold the -i into the adds
  { v2f b0 = v[0][2], b1 = w8_1(v[1][2]), y2 = v[2][2], y3 = w8_1(v[3][2]);
    v2f t0 = add_mi(b0, y2), t1 = sub_mi(b0, y2);
    v2f t2 = add_mi(b1, y3), t3 = sub_mi(b1, y3);
    x[2] = t0 + t2; x[10] = t0 - t2; x[6] = add_mi(t1, t3); x[14] = sub_mi(t1, t3); }
  // c = 3: W16^3, W16^6 = (-i) W16^2, W16^9 = -W16^1
  { v2f b0 = v[0][3], b1 = w16_3(v[1][3]), y2 = w8_1(v[2][3]), u3 = w16_1(v[3][3]);
    v2f t0 = add_mi(b0, y2), t1 = sub_mi(b0, y2);
    v2f t2 = b1 - u3, t3 = b1 + u3;
    x[3] = t0 + t2; x[11] = t0 - t2; x[7] = add_mi(t1, t3); x[15] = sub_mi(t1, t3); }
}

// even half of a DFT16: X[2m] = DFT8(u[n] + u[n+8])
__device__ __forceinline__ void dft16_even(const v2f (&u)[16], v2f (&o)[8]) {
#pragma unroll
  for (int n = 0; n < 8; ++n) o[n] = u[n] + u[n + 8];
  dft8(o);
}

// odd half of a DFT16: X[2m+1] = DFT8((u[n] - u[n+8]) W16^n)
__device__ __forceinline__ void dft16_odd(const v2f (&u)[16], v2f (&o)[8]) {
  o[0] = u[0] - u[8];
  o[1] = w16_1(u[1] - u[9]);
  o[2] = w8_1(u[2] - u[10]);
  o[3] = w16_3(u[3] - u[11]);
  o[4] = u[4] - u[12];            // x (-i): folded into dft8<true>
  o[5] = w16_5(u[5] - u[13]);
  o[6] = w8_1(u[6] - u[14]);      // W16^6 = (-i) W16^2: folded
  o[7] = w16_7(u[7] - u[15]);
  dft8<true>(o);
}

}  // namespace pk
}  // namespace vad
