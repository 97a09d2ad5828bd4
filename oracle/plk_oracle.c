/*
 * plk_oracle.c — CPU restatement of the dusk-plonk hot path. TEST INFRASTRUCTURE ONLY:
 * used by tests/ (as the checker), __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg (timed as the "restated reference CPU path"). The product library
 * (dusk-plonk_amd/libplk.so) never links or calls this file.
 *
 * Independent of the product implementation on purpose: 64-bit limbs with unsigned
 * __int128 (the product uses 32-bit limbs), Jacobian coordinates for G1 (the product uses
 * XYZZ), bit-reversal + iterative butterflies for the NTT (the product uses Stockham
 * passes), unsigned-window Pippenger with per-window doubling (the product uses a signed,
 * precomputed fixed-base table). It is itself cross-checked against oracle/pyref.py (pure
 * Python big ints) and the reference's in-tree known answers in tests/test_oracle.py.
 *
 * Follows (reference call sites; the algorithms live in un-vendored crates):
 *   Fr Montgomery R = 2^256 ......... /root/reference/src/lib.rs:583-588
 *   Fft::{dft,idft,coset_dft,coset_idft}, elements[i] = w^i
 *                                  ... src/permutation.rs:148,194-197,232; src/prover.rs:121-124;
 *                                      src/prover/quotient_poly.rs:54-58,115,145,237,271
 *   compute_vanishing_poly_over_coset  src/key.rs:291
 *   PlonkParams::commit = MSM over the SRS prefix
 *                                  ... src/prover.rs:133-136,194,262-265,440,452; src/key.rs:138-159
 *
 * Parallelism mirrors the reference's rayon pool with OpenMP over all host cores; every
 * entry point takes `threads` (0 = all).
 */
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------------ Fr (4x64) */
static const uint64_t FR_P[4] = {0xffffffff00000001ull, 0x53bda402fffe5bfeull,
                                 0x3339d80809a1d805ull, 0x73eda753299d7d48ull};
static const uint64_t FR_INV = 0xfffffffeffffffffull;
static const uint64_t FR_ONE[4] = {0x00000001fffffffeull, 0x5884b7fa00034802ull,
                                   0x998c4fefecbc4ff5ull, 0x1824b159acc5056full};
static const uint64_t FR_R2[4] = {0xc999e990f3f29c6dull, 0x2b6cedcb87925c23ull,
                                  0x05d314967254398full, 0x0748d9d99f59ff11ull};
/* ROOT_OF_UNITY = 7^((r-1)/2^32), canonical */
static const uint64_t FR_ROOT[4] = {0x3829971f439f0d2bull, 0xb63683508c2280b9ull,
                                    0xd09b681922c813b4ull, 0x16a2a19edfe81f20ull};

/* ------------------------------------------------------------------------ Fp (6x64) */
static const uint64_t FP_P[6] = {0xb9feffffffffaaabull, 0x1eabfffeb153ffffull,
                                 0x6730d2a0f6b0f624ull, 0x64774b84f38512bfull,
                                 0x4b1ba7b6434bacd7ull, 0x1a0111ea397fe69aull};
static const uint64_t FP_INV = 0x89f3fffcfffcfffdull;
static const uint64_t FP_ONE[6] = {0x760900000002fffdull, 0xebf4000bc40c0002ull,
                                   0x5f48985753c758baull, 0x77ce585370525745ull,
                                   0x5c071a97a256ec6dull, 0x15f65ec3fa80e493ull};

/* generic n-limb helpers (n = 4 or 6) */
static int geq(const uint64_t* a, const uint64_t* p, int n) {
  for (int i = n - 1; i >= 0; --i) {
    if (a[i] > p[i]) return 1;
    if (a[i] < p[i]) return 0;
  }
  return 1;
}
static void sub_n(uint64_t* r, const uint64_t* a, const uint64_t* b, int n) {
  uint64_t br = 0;
  for (int i = 0; i < n; ++i) {
    u128 t = (u128)a[i] - b[i] - br;
    r[i] = (uint64_t)t;
    br = (uint64_t)(t >> 127);
  }
}
static void addm(uint64_t* r, const uint64_t* a, const uint64_t* b, const uint64_t* p, int n) {
  uint64_t c = 0, t[6];
  for (int i = 0; i < n; ++i) {
    u128 s = (u128)a[i] + b[i] + c;
    t[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
  if (c || geq(t, p, n)) sub_n(t, t, p, n);
  memcpy(r, t, 8 * n);
}
static void subm(uint64_t* r, const uint64_t* a, const uint64_t* b, const uint64_t* p, int n) {
  uint64_t t[6];
  uint64_t br = 0;
  for (int i = 0; i < n; ++i) {
    u128 s = (u128)a[i] - b[i] - br;
    t[i] = (uint64_t)s;
    br = (uint64_t)(s >> 127);
  }
  if (br) {
    uint64_t c = 0;
    for (int i = 0; i < n; ++i) {
      u128 s = (u128)t[i] + p[i] + c;
      t[i] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
  }
  memcpy(r, t, 8 * n);
}
/* separated operand scanning: full 2n-limb product, then n Montgomery reduction rounds */
static void mulm(uint64_t* r, const uint64_t* a, const uint64_t* b, const uint64_t* p,
                 uint64_t pinv, int n) {
  uint64_t t[13] = {0};
  for (int i = 0; i < n; ++i) {
    uint64_t c = 0;
    for (int j = 0; j < n; ++j) {
      u128 s = (u128)a[i] * b[j] + t[i + j] + c;
      t[i + j] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    t[i + n] = c;
  }
  for (int i = 0; i < n; ++i) {
    uint64_t m = t[i] * pinv, c = 0;
    for (int j = 0; j < n; ++j) {
      u128 s = (u128)m * p[j] + t[i + j] + c;
      t[i + j] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    for (int k = i + n; k < 2 * n + 1 && c; ++k) {
      u128 s = (u128)t[k] + c;
      t[k] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
  }
  uint64_t res[6];
  memcpy(res, t + n, 8 * n);
  if (t[2 * n] || geq(res, p, n)) sub_n(res, res, p, n);
  memcpy(r, res, 8 * n);
}

#define FR_MUL(r, a, b) mulm(r, a, b, FR_P, FR_INV, 4)
#define FR_ADD(r, a, b) addm(r, a, b, FR_P, 4)
#define FR_SUB(r, a, b) subm(r, a, b, FR_P, 4)
#define FP_MUL(r, a, b) mulm(r, a, b, FP_P, FP_INV, 6)
#define FP_ADD(r, a, b) addm(r, a, b, FP_P, 6)
#define FP_SUB(r, a, b) subm(r, a, b, FP_P, 6)

static void fr_pow(uint64_t* r, const uint64_t* a, const uint64_t* e, int ewords) {
  uint64_t acc[4];
  memcpy(acc, FR_ONE, 32);
  for (int w = ewords - 1; w >= 0; --w)
    for (int b = 63; b >= 0; --b) {
      FR_MUL(acc, acc, acc);
      if ((e[w] >> b) & 1) FR_MUL(acc, acc, a);
    }
  memcpy(r, acc, 32);
}
static void fr_inv(uint64_t* r, const uint64_t* a) {
  uint64_t e[4];
  uint64_t two[4] = {2, 0, 0, 0};
  sub_n(e, FR_P, two, 4);
  fr_pow(r, a, e, 4);
}
static void fr_to_mont(uint64_t* r, const uint64_t* a) { FR_MUL(r, a, FR_R2); }
static void fr_from_mont(uint64_t* r, const uint64_t* a) {
  uint64_t one[4] = {1, 0, 0, 0};
  FR_MUL(r, a, one);
}
static void fp_inv(uint64_t* r, const uint64_t* a) {
  uint64_t e[6], two[6] = {2, 0, 0, 0, 0, 0}, acc[6];
  sub_n(e, FP_P, two, 6);
  memcpy(acc, FP_ONE, 48);
  for (int w = 5; w >= 0; --w)
    for (int b = 63; b >= 0; --b) {
      FP_MUL(acc, acc, acc);
      if ((e[w] >> b) & 1) FP_MUL(acc, acc, a);
    }
  memcpy(r, acc, 48);
}

/* ---------------------------------------------------------------------- exported Fr */
void orc_fr_mul(const uint64_t* a, const uint64_t* b, uint64_t* r) { FR_MUL(r, a, b); }
void orc_fr_add(const uint64_t* a, const uint64_t* b, uint64_t* r) { FR_ADD(r, a, b); }
void orc_fr_sub(const uint64_t* a, const uint64_t* b, uint64_t* r) { FR_SUB(r, a, b); }
void orc_fr_inv(const uint64_t* a, uint64_t* r) { fr_inv(r, a); }
void orc_fp_mul(const uint64_t* a, const uint64_t* b, uint64_t* r) { FP_MUL(r, a, b); }

/* w_k in Montgomery form */
void orc_fr_omega(uint32_t log_n, uint64_t* out) {
  uint64_t w[4];
  fr_to_mont(w, FR_ROOT);
  for (uint32_t s = log_n; s < 32; ++s) FR_MUL(w, w, w);
  memcpy(out, w, 32);
}

static void fr_from_u64(uint64_t* r, uint64_t v) {
  uint64_t c[4] = {v, 0, 0, 0};
  fr_to_mont(r, c);
}

/* ---------------------------------------------------------------------- NTT */
static uint64_t bitrev64(uint64_t x, uint32_t bits) {
  uint64_t r = 0;
  for (uint32_t i = 0; i < bits; ++i) r |= ((x >> i) & 1) << (bits - 1 - i);
  return r;
}

/* Fft::elements: out[i] = w^i */
void orc_elements(uint32_t log_n, uint64_t* out, int threads) {
  const uint64_t n = 1ull << log_n;
  uint64_t w[4];
  orc_fr_omega(log_n, w);
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel
  {
    const int nt = omp_get_num_threads(), id = omp_get_thread_num();
    const uint64_t per = (n + nt - 1) / nt, lo = id * per, hi = lo + per < n ? lo + per : n;
    if (lo < hi) {
      uint64_t x[4], e[1] = {lo};
      fr_pow(x, w, e, 1);
      for (uint64_t i = lo; i < hi; ++i) {
        memcpy(out + 4 * i, x, 32);
        FR_MUL(x, x, w);
      }
    }
  }
}

/*
 * In-place NTT on n = 2^log_n Montgomery Fr values (data[len_in..n) must already be zero).
 * dir = +1 forward (dft/coset_dft), -1 inverse (idft/coset_idft); coset uses g = 7.
 */
int orc_ntt(uint64_t* data, uint32_t log_n, int dir, int coset, int threads) {
  const uint64_t n = 1ull << log_n;
  if (threads > 0) omp_set_num_threads(threads);
  uint64_t w[4], g[4];
  orc_fr_omega(log_n, w);
  if (dir < 0) fr_inv(w, w);
  fr_from_u64(g, 7);
  if (coset && dir > 0) {
#pragma omp parallel
    {
      const int nt = omp_get_num_threads(), id = omp_get_thread_num();
      const uint64_t per = (n + nt - 1) / nt, lo = id * per, hi = lo + per < n ? lo + per : n;
      if (lo < hi) {
        uint64_t x[4], e[1] = {lo};
        fr_pow(x, g, e, 1);
        for (uint64_t i = lo; i < hi; ++i) {
          FR_MUL(data + 4 * i, data + 4 * i, x);
          FR_MUL(x, x, g);
        }
      }
    }
  }
  /* bit-reversal permutation */
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)n; ++i) {
    uint64_t j = bitrev64((uint64_t)i, log_n);
    if ((uint64_t)i < j) {
      uint64_t t[4];
      memcpy(t, data + 4 * i, 32);
      memcpy(data + 4 * i, data + 4 * j, 32);
      memcpy(data + 4 * j, t, 32);
    }
  }
  /* twiddles for the largest stage: tw[i] = w^i, i < n/2 */
  uint64_t* tw = (uint64_t*)malloc(sizeof(uint64_t) * 4 * (n / 2 + 1));
  if (!tw) return 1;
  if (n >= 2) {
#pragma omp parallel
    {
      const int nt = omp_get_num_threads(), id = omp_get_thread_num();
      const uint64_t h = n / 2;
      const uint64_t per = (h + nt - 1) / nt, lo = id * per, hi = lo + per < h ? lo + per : h;
      if (lo < hi) {
        uint64_t x[4], e[1] = {lo};
        fr_pow(x, w, e, 1);
        for (uint64_t i = lo; i < hi; ++i) {
          memcpy(tw + 4 * i, x, 32);
          FR_MUL(x, x, w);
        }
      }
    }
  }
  for (uint32_t s = 1; s <= log_n; ++s) {
    const uint64_t m = 1ull << s, half = m >> 1, step = n >> s;
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < (int64_t)(n / 2); ++b) {
      const uint64_t grp = (uint64_t)b / half, r = (uint64_t)b % half;
      const uint64_t i = grp * m + r, j = i + half;
      uint64_t t[4], u[4];
      FR_MUL(t, data + 4 * j, tw + 4 * (r * step));
      memcpy(u, data + 4 * i, 32);
      FR_ADD(data + 4 * i, u, t);
      FR_SUB(data + 4 * j, u, t);
    }
  }
  free(tw);
  if (dir < 0) {
    uint64_t ninv[4], gi[4];
    fr_from_u64(ninv, n);
    fr_inv(ninv, ninv);
    fr_inv(gi, g);
#pragma omp parallel
    {
      const int nt = omp_get_num_threads(), id = omp_get_thread_num();
      const uint64_t per = (n + nt - 1) / nt, lo = id * per, hi = lo + per < n ? lo + per : n;
      if (lo < hi) {
        uint64_t x[4], e[1] = {lo};
        if (coset) {
          fr_pow(x, gi, e, 1);
          FR_MUL(x, x, ninv);
        } else {
          memcpy(x, ninv, 32);
        }
        for (uint64_t i = lo; i < hi; ++i) {
          FR_MUL(data + 4 * i, data + 4 * i, x);
          if (coset) FR_MUL(x, x, gi);
        }
      }
    }
  }
  return 0;
}

/* v_h[i] = (g w^i)^deg - 1 on the 2^log_n domain (key.rs:291) */
void orc_vanishing(uint32_t log_n, uint64_t deg, uint64_t* out) {
  const uint64_t n = 1ull << log_n;
  uint64_t w[4], g[4], gd[4], wd[4], x[4], e[1] = {deg};
  orc_fr_omega(log_n, w);
  fr_from_u64(g, 7);
  fr_pow(gd, g, e, 1);
  fr_pow(wd, w, e, 1);
  memcpy(x, gd, 32);
  for (uint64_t i = 0; i < n; ++i) {
    FR_SUB(out + 4 * i, x, FR_ONE);
    FR_MUL(x, x, wd);
  }
}

/* ---------------------------------------------------------------------- G1 (Jacobian) */
typedef struct {
  uint64_t X[6], Y[6], Z[6];
} jac;

static int fp_is_zero(const uint64_t* a) { return !(a[0] | a[1] | a[2] | a[3] | a[4] | a[5]); }
static void jac_set_inf(jac* p) {
  memcpy(p->X, FP_ONE, 48);
  memcpy(p->Y, FP_ONE, 48);
  memset(p->Z, 0, 48);
}

/* dbl-2009-l */
static void jac_dbl(jac* r, const jac* p) {
  if (fp_is_zero(p->Z)) {
    *r = *p;
    return;
  }
  uint64_t A[6], B[6], C[6], D[6], E[6], F[6], t[6], X3[6], Y3[6], Z3[6];
  FP_MUL(A, p->X, p->X);
  FP_MUL(B, p->Y, p->Y);
  FP_MUL(C, B, B);
  FP_ADD(t, p->X, B);
  FP_MUL(t, t, t);
  FP_SUB(t, t, A);
  FP_SUB(t, t, C);
  FP_ADD(D, t, t);
  FP_ADD(E, A, A);
  FP_ADD(E, E, A);
  FP_MUL(F, E, E);
  FP_SUB(X3, F, D);
  FP_SUB(X3, X3, D);
  FP_SUB(t, D, X3);
  FP_MUL(Y3, E, t);
  FP_ADD(t, C, C);
  FP_ADD(t, t, t);
  FP_ADD(t, t, t);
  FP_SUB(Y3, Y3, t);
  FP_MUL(Z3, p->Y, p->Z);
  FP_ADD(Z3, Z3, Z3);
  memcpy(r->X, X3, 48);
  memcpy(r->Y, Y3, 48);
  memcpy(r->Z, Z3, 48);
}

/* madd-2007-bl: p + (x2, y2) affine */
static void jac_add_aff(jac* r, const jac* p, const uint64_t* x2, const uint64_t* y2) {
  if (fp_is_zero(p->Z)) {
    memcpy(r->X, x2, 48);
    memcpy(r->Y, y2, 48);
    memcpy(r->Z, FP_ONE, 48);
    return;
  }
  uint64_t Z1Z1[6], U2[6], S2[6], H[6], HH[6], I[6], J[6], rr[6], V[6], t[6];
  FP_MUL(Z1Z1, p->Z, p->Z);
  FP_MUL(U2, x2, Z1Z1);
  FP_MUL(S2, y2, p->Z);
  FP_MUL(S2, S2, Z1Z1);
  FP_SUB(H, U2, p->X);
  FP_SUB(rr, S2, p->Y);
  if (fp_is_zero(H)) {
    if (fp_is_zero(rr)) {
      jac q;
      memcpy(q.X, x2, 48);
      memcpy(q.Y, y2, 48);
      memcpy(q.Z, FP_ONE, 48);
      jac_dbl(r, &q);
    } else {
      jac_set_inf(r);
    }
    return;
  }
  FP_MUL(HH, H, H);
  FP_ADD(I, HH, HH);
  FP_ADD(I, I, I);
  FP_MUL(J, H, I);
  FP_ADD(rr, rr, rr);
  FP_MUL(V, p->X, I);
  jac o;
  FP_MUL(o.X, rr, rr);
  FP_SUB(o.X, o.X, J);
  FP_SUB(o.X, o.X, V);
  FP_SUB(o.X, o.X, V);
  FP_SUB(t, V, o.X);
  FP_MUL(o.Y, rr, t);
  FP_MUL(t, p->Y, J);
  FP_ADD(t, t, t);
  FP_SUB(o.Y, o.Y, t);
  FP_ADD(t, p->Z, H);
  FP_MUL(t, t, t);
  FP_SUB(t, t, Z1Z1);
  FP_SUB(o.Z, t, HH);
  *r = o;
}

/* add-2007-bl: general */
static void jac_add(jac* r, const jac* p, const jac* q) {
  if (fp_is_zero(p->Z)) {
    *r = *q;
    return;
  }
  if (fp_is_zero(q->Z)) {
    *r = *p;
    return;
  }
  uint64_t Z1Z1[6], Z2Z2[6], U1[6], U2[6], S1[6], S2[6], H[6], I[6], J[6], rr[6], V[6], t[6];
  FP_MUL(Z1Z1, p->Z, p->Z);
  FP_MUL(Z2Z2, q->Z, q->Z);
  FP_MUL(U1, p->X, Z2Z2);
  FP_MUL(U2, q->X, Z1Z1);
  FP_MUL(S1, p->Y, q->Z);
  FP_MUL(S1, S1, Z2Z2);
  FP_MUL(S2, q->Y, p->Z);
  FP_MUL(S2, S2, Z1Z1);
  FP_SUB(H, U2, U1);
  FP_SUB(rr, S2, S1);
  if (fp_is_zero(H)) {
    if (fp_is_zero(rr)) {
      jac_dbl(r, p);
    } else {
      jac_set_inf(r);
    }
    return;
  }
  FP_ADD(I, H, H);
  FP_MUL(I, I, I);
  FP_MUL(J, H, I);
  FP_ADD(rr, rr, rr);
  FP_MUL(V, U1, I);
  jac o;
  FP_MUL(o.X, rr, rr);
  FP_SUB(o.X, o.X, J);
  FP_SUB(o.X, o.X, V);
  FP_SUB(o.X, o.X, V);
  FP_SUB(t, V, o.X);
  FP_MUL(o.Y, rr, t);
  FP_MUL(t, S1, J);
  FP_ADD(t, t, t);
  FP_SUB(o.Y, o.Y, t);
  FP_ADD(t, p->Z, q->Z);
  FP_MUL(t, t, t);
  FP_SUB(t, t, Z1Z1);
  FP_SUB(t, t, Z2Z2);
  FP_MUL(o.Z, t, H);
  *r = o;
}

/* canonical affine, 13-word ABI layout */
static void jac_to_abi(const jac* p, uint64_t* out) {
  memset(out, 0, 13 * 8);
  if (fp_is_zero(p->Z)) {
    out[12] = 1;
    return;
  }
  uint64_t zi[6], zi2[6], zi3[6];
  fp_inv(zi, p->Z);
  FP_MUL(zi2, zi, zi);
  FP_MUL(zi3, zi2, zi);
  FP_MUL(out, p->X, zi2);
  FP_MUL(out + 6, p->Y, zi3);
}

/*
 * MSM: out = sum scalars[i] * points[i]; points in the 13-word ABI layout (Montgomery Fp
 * + infinity flag), scalars Montgomery Fr. Unsigned-window Pippenger, c ~ ln(n), windows
 * processed in parallel, then the per-window doubling chain.
 */
int orc_msm(const uint64_t* points, const uint64_t* scalars, size_t n, uint64_t* out,
            int threads) {
  if (threads > 0) omp_set_num_threads(threads);
  uint32_t c = 1;
  while ((1ull << (c + 1)) <= (uint64_t)(n ? n : 1) && c < 16) ++c; /* ~log2 n */
  c = c > 3 ? c - 2 : 2;                                             /* ~ln n */
  const uint32_t W = (255 + c - 1) / c;
  uint64_t* sc = (uint64_t*)malloc(32 * (n ? n : 1));
  jac* win = (jac*)malloc(sizeof(jac) * W);
  if (!sc || !win) return 1;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)n; ++i) fr_from_mont(sc + 4 * i, scalars + 4 * i);
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t w = 0; w < (int64_t)W; ++w) {
    const uint64_t nb = 1ull << c;
    jac* bk = (jac*)malloc(sizeof(jac) * nb);
    for (uint64_t b = 0; b < nb; ++b) jac_set_inf(&bk[b]);
    const uint32_t o = (uint32_t)w * c;
    for (size_t i = 0; i < n; ++i) {
      const uint64_t* pt = points + 13 * i;
      if (pt[12]) continue;
      const uint32_t wd = o >> 6, sh = o & 63;
      u128 two = sc[4 * i + wd];
      if (wd + 1 < 4) two |= (u128)sc[4 * i + wd + 1] << 64;
      const uint64_t d = (uint64_t)(two >> sh) & (nb - 1);
      if (d) jac_add_aff(&bk[d], &bk[d], pt, pt + 6);
    }
    jac run, acc;
    jac_set_inf(&run);
    jac_set_inf(&acc);
    for (uint64_t b = nb - 1; b >= 1; --b) {
      jac_add(&run, &run, &bk[b]);
      jac_add(&acc, &acc, &run);
    }
    win[w] = acc;
    free(bk);
  }
  jac total;
  jac_set_inf(&total);
  for (int64_t w = (int64_t)W - 1; w >= 0; --w) {
    for (uint32_t k = 0; k < c; ++k) jac_dbl(&total, &total);
    jac_add(&total, &total, &win[w]);
  }
  jac_to_abi(&total, out);
  free(sc);
  free(win);
  return 0;
}

/* [k]P by double-and-add, P affine ABI, k Montgomery Fr -> ABI */
void orc_g1_mul(const uint64_t* pt, const uint64_t* k_mont, uint64_t* out) {
  uint64_t k[4];
  fr_from_mont(k, k_mont);
  jac acc;
  jac_set_inf(&acc);
  if (!pt[12])
    for (int b = 255; b >= 0; --b) {
      jac_dbl(&acc, &acc);
      if ((k[b >> 6] >> (b & 63)) & 1) jac_add_aff(&acc, &acc, pt, pt + 6);
    }
  jac_to_abi(&acc, out);
}

/* PlonkParams::setup restated: out[i] = [tau^i] G1 (ABI layout), tau Montgomery Fr */
void orc_srs(const uint64_t* tau_mont, size_t n, uint64_t* out, int threads) {
  static const uint64_t GX[6] = {0xfb3af00adb22c6bbull, 0x6c55e83ff97a1aefull,
                                 0xa14e3a3f171bac58ull, 0xc3688c4f9774b905ull,
                                 0x2695638c4fa9ac0full, 0x17f1d3a73197d794ull};
  static const uint64_t GY[6] = {0x0caa232946c5e7e1ull, 0xd03cc744a2888ae4ull,
                                 0x00db18cb2c04b3edull, 0xfcf5e095d5d00af6ull,
                                 0xa09e30ed741d8ae4ull, 0x08b3f481e3aaa0f1ull};
  static const uint64_t FP_R2[6] = {0xf4df1f341c341746ull, 0x0a76e6a609d104f1ull,
                                    0x8de5476c4c95b6d5ull, 0x67eb88a9939d83c0ull,
                                    0x9a793e85b519952dull, 0x11988fe592cae3aaull};
  uint64_t gen[13] = {0};
  FP_MUL(gen, GX, FP_R2);
  FP_MUL(gen + 6, GY, FP_R2);
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t i = 0; i < (int64_t)n; ++i) {
    uint64_t t[4], e[1] = {(uint64_t)i};
    fr_pow(t, tau_mont, e, 1);
    orc_g1_mul(gen, t, out + 13 * i);
  }
}
