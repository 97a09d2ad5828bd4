// g1.hpp — BLS12-381 G1 (y^2 = x^3 + 4 over Fp) point arithmetic for the MSM.
//
// Restates the group law of the un-vendored `bls-12-381` crate that
// `msm_curve_addition` / `PlonkParams::commit` run on. Accumulators use extended
// Jacobian "XYZZ" coordinates (x = X/ZZ, y = Y/ZZZ, ZZ^3 = ZZZ^2): a mixed add with an
// affine base costs 8M + 2S, with no doubling special case on the hot path except the
// exact-equality branch. Formulas: EFD g1p/shortw/xyzz (madd-2008-s, add-2008-s,
// dbl-2008-s-1, mdbl-2008-s-1), a = 0.
#pragma once
#include "ff.hpp"

namespace plk {

struct alignas(16) G1Affine {
  Fp x, y;  // infinity is carried separately (flag or sentinel), never as coordinates
};

struct G1xyzz {
  Fp X, Y, ZZ, ZZZ;  // ZZ == 0  <=>  point at infinity
};

PLK_HD G1xyzz xyzz_infinity() {
  G1xyzz r;
  r.X = fe_one<FpCfg>();
  r.Y = fe_one<FpCfg>();
  r.ZZ = fe_zero<FpCfg>();
  r.ZZZ = fe_zero<FpCfg>();
  return r;
}

PLK_HD bool xyzz_is_inf(const G1xyzz& p) { return fe_is_zero(p.ZZ); }

PLK_HD G1xyzz xyzz_from_affine(const G1Affine& a) {
  G1xyzz r;
  r.X = a.x;
  r.Y = a.y;
  r.ZZ = fe_one<FpCfg>();
  r.ZZZ = fe_one<FpCfg>();
  return r;
}

PLK_HD G1xyzz xyzz_neg(const G1xyzz& p) {
  G1xyzz r = p;
  r.Y = fe_neg(p.Y);
  return r;
}

// dbl-2008-s-1
PLK_HD G1xyzz xyzz_dbl(const G1xyzz& p) {
  if (xyzz_is_inf(p)) return p;
  Fp U = fe_dbl(p.Y);
  Fp V = fe_sqr(U);
  Fp W = fe_mul(U, V);
  Fp S = fe_mul(p.X, V);
  Fp X2 = fe_sqr(p.X);
  Fp M = fe_add(fe_dbl(X2), X2);
  G1xyzz r;
  r.X = fe_sub(fe_sqr(M), fe_dbl(S));
  r.Y = fe_sub(fe_mul(M, fe_sub(S, r.X)), fe_mul(W, p.Y));
  r.ZZ = fe_mul(V, p.ZZ);
  r.ZZZ = fe_mul(W, p.ZZZ);
  return r;
}

// mdbl-2008-s-1: double an affine point into XYZZ
PLK_HD G1xyzz xyzz_dbl_affine(const Fp& x, const Fp& y) {
  Fp U = fe_dbl(y);
  Fp V = fe_sqr(U);
  Fp W = fe_mul(U, V);
  Fp S = fe_mul(x, V);
  Fp X2 = fe_sqr(x);
  Fp M = fe_add(fe_dbl(X2), X2);
  G1xyzz r;
  r.X = fe_sub(fe_sqr(M), fe_dbl(S));
  r.Y = fe_sub(fe_mul(M, fe_sub(S, r.X)), fe_mul(W, y));
  r.ZZ = V;
  r.ZZZ = W;
  return r;
}

// madd-2008-s: p + (x2, y2), the affine operand is never infinity
PLK_HD G1xyzz xyzz_add_affine(const G1xyzz& p, const Fp& x2, const Fp& y2) {
  if (xyzz_is_inf(p)) {
    G1xyzz r;
    r.X = x2;
    r.Y = y2;
    r.ZZ = fe_one<FpCfg>();
    r.ZZZ = fe_one<FpCfg>();
    return r;
  }
  Fp U2 = fe_mul(x2, p.ZZ);
  Fp S2 = fe_mul(y2, p.ZZZ);
  Fp P = fe_sub(U2, p.X);
  Fp R = fe_sub(S2, p.Y);
  if (fe_is_zero(P)) {
    if (fe_is_zero(R)) return xyzz_dbl_affine(x2, y2);
    return xyzz_infinity();
  }
  Fp PP = fe_sqr(P);
  Fp PPP = fe_mul(P, PP);
  Fp Q = fe_mul(p.X, PP);
  G1xyzz r;
  r.X = fe_sub(fe_sub(fe_sqr(R), PPP), fe_dbl(Q));
  r.Y = fe_sub(fe_mul(R, fe_sub(Q, r.X)), fe_mul(p.Y, PPP));
  r.ZZ = fe_mul(p.ZZ, PP);
  r.ZZZ = fe_mul(p.ZZZ, PPP);
  return r;
}

// add-2008-s: general XYZZ + XYZZ
PLK_HD G1xyzz xyzz_add(const G1xyzz& p, const G1xyzz& q) {
  if (xyzz_is_inf(p)) return q;
  if (xyzz_is_inf(q)) return p;
  Fp U1 = fe_mul(p.X, q.ZZ);
  Fp U2 = fe_mul(q.X, p.ZZ);
  Fp S1 = fe_mul(p.Y, q.ZZZ);
  Fp S2 = fe_mul(q.Y, p.ZZZ);
  Fp P = fe_sub(U2, U1);
  Fp R = fe_sub(S2, S1);
  if (fe_is_zero(P)) {
    if (fe_is_zero(R)) return xyzz_dbl(p);
    return xyzz_infinity();
  }
  Fp PP = fe_sqr(P);
  Fp PPP = fe_mul(P, PP);
  Fp Q = fe_mul(U1, PP);
  G1xyzz r;
  r.X = fe_sub(fe_sub(fe_sqr(R), PPP), fe_dbl(Q));
  r.Y = fe_sub(fe_mul(R, fe_sub(Q, r.X)), fe_mul(S1, PPP));
  r.ZZ = fe_mul(fe_mul(p.ZZ, q.ZZ), PP);
  r.ZZZ = fe_mul(fe_mul(p.ZZZ, q.ZZZ), PPP);
  return r;
}

// XYZZ -> affine; returns false for infinity. One field inversion (of ZZZ):
// 1/ZZ = (ZZ / ZZZ)^2 because ZZ^3 = ZZZ^2.
PLK_HD bool xyzz_to_affine(const G1xyzz& p, Fp& x, Fp& y) {
  if (xyzz_is_inf(p)) {
    x = fe_zero<FpCfg>();
    y = fe_zero<FpCfg>();
    return false;
  }
  Fp u = fe_inv(p.ZZZ);
  Fp zzinv = fe_sqr(fe_mul(p.ZZ, u));
  x = fe_mul(p.X, zzinv);
  y = fe_mul(p.Y, u);
  return true;
}

}  // namespace plk
