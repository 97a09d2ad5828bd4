/*
 * plk_prover_oracle.c — CPU restatement of PlonkKey::compile + Prover::create_proof.
 * TEST INFRASTRUCTURE ONLY: the byte-level checker of the GPU prover (tests/) and the
 * timed "restated reference CPU path" of the full prover (bench.py cpu_baseline). The
 * product library never links or calls this file.
 *
 * It includes plk_oracle.c (field, NTT, MSM restatements) and restates, in the
 * reference's own order of operations and cost structure:
 *   key compile ..... src/key.rs:63-327 (selector idft :121-131, commitments :138-159 with
 *                     unwrap_or_default for selectors, 8n coset evaluations :220-245,
 *                     v_h over the coset :291), src/permutation.rs:108-168 (sigma =
 *                     next wire in insertion order, Lagrange encodings w^i {1,K1,K2,K3})
 *   create_proof .... src/prover.rs:67-474 (transcript order, blinding of wires with 2
 *                     and z with 3 scalars, t split :252-259, openings :407-452)
 *   grand product ... src/permutation.rs:205-300 (dft of sigmas, per-gate num/den, one
 *                     inversion per gate, sequential prefix product)
 *   quotient ........ src/prover/quotient_poly.rs (8n coset, 8 wrap-around rows, the
 *                     sequential widget loop, parallel permutation loop, one inversion of
 *                     v_h per point in a sequential loop)
 *   linearisation ... src/prover/linearization_poly.rs (evaluations, arithmetic + range +
 *                     permutation linearisers)
 *   transcript ...... merlin (STROBE-128 / Keccak-f[1600]) with dusk-plonk's
 *                     TranscriptProtocol (append_scalar = 32 LE bytes, append_commitment =
 *                     48-byte compressed G1, challenge_scalar = from_bytes_wide of 64
 *                     bytes), restated from the merlin / STROBE specifications; pinned by
 *                     merlin's published test vector (tests/test_transcript.py).
 * Randomness: the blinding scalars come from SplitMix64(seed), 4 words per scalar, top word
 * masked to 255 bits, rejection-sampled below r — the GPU prover consumes the
 * same stream in the same order (a, b, c, d: 2 each; z: 3).
 * Widgets restated: arithmetic, range, logic, fixed-base scalar multiplication and
 * variable-base addition (the latter three from upstream dusk-plonk: parity unpinned).
 */
#include "plk_oracle.c"

#include <time.h>

enum { ORC_OK = 0, ORC_E_ARG = 1, ORC_E_DEGREE = 2, ORC_E_OOM = 4, ORC_E_UNSUPPORTED = 6 };

/* ------------------------------------------------------------------------ helpers */
typedef uint64_t fr_t[4];

static void fr_set(uint64_t* r, const uint64_t* a) { memcpy(r, a, 32); }
static void fr_zero(uint64_t* r) { memset(r, 0, 32); }
static int fr_is_zero(const uint64_t* a) { return !(a[0] | a[1] | a[2] | a[3]); }
static void fr_neg(uint64_t* r, const uint64_t* a) {
  uint64_t z[4] = {0, 0, 0, 0};
  FR_SUB(r, z, a);
}
static void fr_pow_u64(uint64_t* r, const uint64_t* a, uint64_t e) {
  uint64_t w[1] = {e};
  fr_pow(r, a, w, 1);
}
static uint64_t now_ns(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}
static uint64_t* fr_alloc(size_t n) { return (uint64_t*)calloc(n ? n : 1, 32); }

/* Horner evaluation of sum c_i x^i */
static void poly_eval(uint64_t* r, const uint64_t* c, size_t len, const uint64_t* x) {
  uint64_t acc[4] = {0, 0, 0, 0};
  for (size_t i = len; i-- > 0;) {
    FR_MUL(acc, acc, x);
    FR_ADD(acc, acc, c + 4 * i);
  }
  fr_set(r, acc);
}

/* out[0..len) += s * p[0..plen) (out has >= plen entries) */
static void poly_axpy(uint64_t* out, const uint64_t* p, size_t plen, const uint64_t* s) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)plen; ++i) {
    uint64_t t[4];
    FR_MUL(t, p + 4 * i, s);
    FR_ADD(out + 4 * i, out + 4 * i, t);
  }
}

/* poly_commit Coefficients::ruffini: quotient of p(X) by (X - z), length len - 1 */
static void poly_ruffini(uint64_t* q, const uint64_t* c, size_t len, const uint64_t* z) {
  if (len < 2) return;
  uint64_t acc[4] = {0, 0, 0, 0};
  for (size_t k = len - 1; k >= 1; --k) {
    FR_MUL(acc, acc, z);
    FR_ADD(acc, acc, c + 4 * k);
    fr_set(q + 4 * (k - 1), acc);
  }
}

/* ------------------------------------------------------------------------ SplitMix64 */
typedef struct {
  uint64_t s;
} orc_rng;
static uint64_t rng_next(orc_rng* g) {
  g->s += 0x9E3779B97F4A7C15ull;
  uint64_t z = g->s;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static void rng_fr(orc_rng* g, uint64_t* out) {
  for (;;) {
    uint64_t c[4];
    for (int i = 0; i < 4; ++i) c[i] = rng_next(g);
    c[3] &= 0x7fffffffffffffffull;
    if (!geq(c, FR_P, 4)) {
      fr_to_mont(out, c);
      return;
    }
  }
}

/* ------------------------------------------------------------------ merlin transcript */
static const uint64_t KECCAK_RC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
    0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
    0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
/* rotation offsets r[x + 5y] */
static const int KECCAK_ROT[25] = {0,  1,  62, 28, 27, 36, 44, 6,  55, 20, 3,  10, 43,
                                   25, 39, 41, 45, 15, 21, 8,  18, 2,  61, 56, 14};
static uint64_t rotl64(uint64_t x, int n) { return n ? (x << n) | (x >> (64 - n)) : x; }

static void keccak_f1600(uint8_t* bytes) {
  uint64_t A[25], B[25], C[5], D[5];
  for (int i = 0; i < 25; ++i) {
    uint64_t v = 0;
    for (int k = 7; k >= 0; --k) v = (v << 8) | bytes[8 * i + k];
    A[i] = v;
  }
  for (int round = 0; round < 24; ++round) {
    for (int x = 0; x < 5; ++x) C[x] = A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20];
    for (int x = 0; x < 5; ++x) D[x] = C[(x + 4) % 5] ^ rotl64(C[(x + 1) % 5], 1);
    for (int i = 0; i < 25; ++i) A[i] ^= D[i % 5];
    /* rho + pi: B[y + 5*((2x + 3y) % 5)] = rot(A[x + 5y]) */
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y) B[y + 5 * ((2 * x + 3 * y) % 5)] = rotl64(A[x + 5 * y], KECCAK_ROT[x + 5 * y]);
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y)
        A[x + 5 * y] = B[x + 5 * y] ^ (~B[(x + 1) % 5 + 5 * y] & B[(x + 2) % 5 + 5 * y]);
    A[0] ^= KECCAK_RC[round];
  }
  for (int i = 0; i < 25; ++i)
    for (int k = 0; k < 8; ++k) bytes[8 * i + k] = (uint8_t)(A[i] >> (8 * k));
}

enum { ST_I = 1, ST_A = 2, ST_C = 4, ST_T = 8, ST_M = 16, ST_K = 32, ST_R = 166 };
typedef struct {
  uint8_t st[200];
  int pos, pos_begin, cur_flags;
} orc_strobe;

static void strobe_run_f(orc_strobe* s) {
  s->st[s->pos] ^= (uint8_t)s->pos_begin;
  s->st[s->pos + 1] ^= 0x04;
  s->st[ST_R + 1] ^= 0x80;
  keccak_f1600(s->st);
  s->pos = 0;
  s->pos_begin = 0;
}
static void strobe_absorb(orc_strobe* s, const uint8_t* d, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    s->st[s->pos] ^= d[i];
    if (++s->pos == ST_R) strobe_run_f(s);
  }
}
static void strobe_squeeze(orc_strobe* s, uint8_t* d, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    d[i] = s->st[s->pos];
    s->st[s->pos] = 0;
    if (++s->pos == ST_R) strobe_run_f(s);
  }
}
static void strobe_begin_op(orc_strobe* s, int flags, int more) {
  if (more) return; /* continuation of the same operation */
  const uint8_t hdr[2] = {(uint8_t)s->pos_begin, (uint8_t)flags};
  s->pos_begin = s->pos + 1;
  s->cur_flags = flags;
  strobe_absorb(s, hdr, 2);
  if ((flags & (ST_C | ST_K)) && s->pos != 0) strobe_run_f(s);
}
static void strobe_meta_ad(orc_strobe* s, const uint8_t* d, size_t n, int more) {
  strobe_begin_op(s, ST_M | ST_A, more);
  strobe_absorb(s, d, n);
}
static void strobe_ad(orc_strobe* s, const uint8_t* d, size_t n, int more) {
  strobe_begin_op(s, ST_A, more);
  strobe_absorb(s, d, n);
}
static void strobe_prf(orc_strobe* s, uint8_t* d, size_t n, int more) {
  strobe_begin_op(s, ST_I | ST_A | ST_C, more);
  strobe_squeeze(s, d, n);
}
static void strobe_init(orc_strobe* s, const char* label) {
  memset(s, 0, sizeof *s);
  const uint8_t init[6] = {1, ST_R + 2, 1, 0, 1, 96};
  memcpy(s->st, init, 6);
  memcpy(s->st + 6, "STROBEv1.0.2", 12);
  keccak_f1600(s->st);
  strobe_meta_ad(s, (const uint8_t*)label, strlen(label), 0);
}

typedef struct {
  orc_strobe s;
} orc_transcript;

static void tr_append_message(orc_transcript* t, const char* label, const uint8_t* msg, size_t n) {
  const uint8_t len[4] = {(uint8_t)n, (uint8_t)(n >> 8), (uint8_t)(n >> 16), (uint8_t)(n >> 24)};
  strobe_meta_ad(&t->s, (const uint8_t*)label, strlen(label), 0);
  strobe_meta_ad(&t->s, len, 4, 1);
  strobe_ad(&t->s, msg, n, 0);
}
static void tr_init(orc_transcript* t, const uint8_t* label, size_t n) {
  strobe_init(&t->s, "Merlin v1.0");
  tr_append_message(t, "dom-sep", label, n);
}
static void tr_append_u64(orc_transcript* t, const char* label, uint64_t x) {
  uint8_t b[8];
  for (int i = 0; i < 8; ++i) b[i] = (uint8_t)(x >> (8 * i));
  tr_append_message(t, label, b, 8);
}
static void tr_challenge_bytes(orc_transcript* t, const char* label, uint8_t* out, size_t n) {
  const uint8_t len[4] = {(uint8_t)n, (uint8_t)(n >> 8), (uint8_t)(n >> 16), (uint8_t)(n >> 24)};
  strobe_meta_ad(&t->s, (const uint8_t*)label, strlen(label), 0);
  strobe_meta_ad(&t->s, len, 4, 1);
  strobe_prf(&t->s, out, n, 0);
}
/* TranscriptProtocol::append_scalar: canonical little-endian 32 bytes */
static void tr_append_scalar(orc_transcript* t, const char* label, const uint64_t* s_mont) {
  uint64_t c[4];
  uint8_t b[32];
  fr_from_mont(c, s_mont);
  for (int i = 0; i < 32; ++i) b[i] = (uint8_t)(c[i / 8] >> (8 * (i % 8)));
  tr_append_message(t, label, b, 32);
}
/* G1 compressed (zkcrypto encoding): big-endian x, flags 0x80 compressed, 0x40 infinity,
 * 0x20 when y is the lexicographically larger root */
static void g1_compress(const uint64_t* p13, uint8_t* out) {
  memset(out, 0, 48);
  if (p13[12]) {
    out[0] = 0xc0;
    return;
  }
  uint64_t x[6], y[6], ny[6], one[6] = {1, 0, 0, 0, 0, 0};
  FP_MUL(x, p13, one);
  FP_MUL(y, p13 + 6, one);
  uint64_t zero[6] = {0, 0, 0, 0, 0, 0};
  FP_SUB(ny, zero, y);
  for (int k = 0; k < 48; ++k) out[47 - k] = (uint8_t)(x[k / 8] >> (8 * (k % 8)));
  int larger = 0;
  for (int i = 5; i >= 0; --i)
    if (y[i] != ny[i]) {
      larger = y[i] > ny[i];
      break;
    }
  out[0] |= 0x80 | (larger ? 0x20 : 0);
}
static void tr_append_commitment(orc_transcript* t, const char* label, const uint64_t* p13) {
  uint8_t b[48];
  g1_compress(p13, b);
  tr_append_message(t, label, b, 48);
}
/* challenge_scalar: Fr::from_bytes_wide(64 bytes) = (lo + hi 2^256) mod r, Montgomery out */
static void tr_challenge_scalar(orc_transcript* t, const char* label, uint64_t* out) {
  uint8_t b[64];
  tr_challenge_bytes(t, label, b, 64);
  uint64_t lo[4] = {0}, hi[4] = {0}, r3[4], a[4], c[4];
  for (int i = 0; i < 32; ++i) {
    lo[i / 8] |= (uint64_t)b[i] << (8 * (i % 8));
    hi[i / 8] |= (uint64_t)b[32 + i] << (8 * (i % 8));
  }
  FR_MUL(r3, FR_R2, FR_R2); /* R^3 */
  FR_MUL(a, lo, FR_R2);     /* lo * R */
  FR_MUL(c, hi, r3);        /* hi * 2^256 * R */
  FR_ADD(out, a, c);
}

/* merlin's published test vector driver: transcript "test protocol", append "some label"
 * = "some data", 32 challenge bytes under "challenge" */
void orc_merlin_test(uint8_t* out32) {
  orc_transcript t;
  tr_init(&t, (const uint8_t*)"test protocol", 13);
  tr_append_message(&t, "some label", (const uint8_t*)"some data", 9);
  tr_challenge_bytes(&t, "challenge", out32, 32);
}

/* -------------------------------------------------------------------- logic widget */
static void fr_small(uint64_t* r, uint64_t v) { fr_from_u64(r, v); }
static void fr_delta(uint64_t* r, const uint64_t* f) { /* f (f - 1)(f - 2)(f - 3) */
  fr_t k, t, u;
  fr_set(u, f);
  fr_small(k, 1);
  FR_SUB(t, f, k);
  FR_MUL(u, u, t);
  fr_small(k, 2);
  FR_SUB(t, f, k);
  FR_MUL(u, u, t);
  fr_small(k, 3);
  FR_SUB(t, f, k);
  FR_MUL(r, u, t);
}
/* dusk-plonk logic gate (zksnarks LogicGate widget, un-vendored): with quads
 * a' = a_next - 4a, b' = b_next - 4b, d' = d_next - 4d and w = c:
 *   D(a') + D(b') k + D(d') k^2 + (w - a'b') k^3 + xor_and(a', b', w, d', q_c) k^4
 * xor_and = 3(a' + b' + d') - 2F + q_c (9d' - 3(a' + b')),
 * F = w (w (4w - 18(a' + b') + 81) + 18(a'^2 + b'^2) - 81(a' + b') + 83) */
static void logic_terms(uint64_t* out, const uint64_t* a, const uint64_t* an, const uint64_t* b,
                        const uint64_t* bn, const uint64_t* w, const uint64_t* d,
                        const uint64_t* dn, const uint64_t* qc, fr_t* lk) {
  fr_t four, qa, qb, qd, t, u, sum, k;
  fr_small(four, 4);
  FR_MUL(t, four, a);
  FR_SUB(qa, an, t);
  FR_MUL(t, four, b);
  FR_SUB(qb, bn, t);
  FR_MUL(t, four, d);
  FR_SUB(qd, dn, t);
  fr_delta(sum, qa);
  fr_delta(t, qb);
  FR_MUL(t, t, lk[1]);
  FR_ADD(sum, sum, t);
  fr_delta(t, qd);
  FR_MUL(t, t, lk[2]);
  FR_ADD(sum, sum, t);
  FR_MUL(t, qa, qb);
  FR_SUB(t, w, t);
  FR_MUL(t, t, lk[3]);
  FR_ADD(sum, sum, t);
  /* F */
  fr_t ab, f;
  FR_ADD(ab, qa, qb);
  fr_small(k, 4);
  FR_MUL(f, k, w);
  fr_small(k, 18);
  FR_MUL(t, k, ab);
  FR_SUB(f, f, t);
  fr_small(k, 81);
  FR_ADD(f, f, k);
  FR_MUL(f, f, w);
  FR_MUL(t, qa, qa);
  FR_MUL(u, qb, qb);
  FR_ADD(t, t, u);
  fr_small(k, 18);
  FR_MUL(t, t, k);
  FR_ADD(f, f, t);
  fr_small(k, 81);
  FR_MUL(t, k, ab);
  FR_SUB(f, f, t);
  fr_small(k, 83);
  FR_ADD(f, f, k);
  FR_MUL(f, f, w);
  /* e = 3(a' + b' + d') - 2F ; bb = q_c (9d' - 3(a' + b')) */
  fr_t e, bb;
  FR_ADD(t, ab, qd);
  fr_small(k, 3);
  FR_MUL(e, k, t);
  FR_ADD(t, f, f);
  FR_SUB(e, e, t);
  fr_small(k, 9);
  FR_MUL(bb, k, qd);
  fr_small(k, 3);
  FR_MUL(t, k, ab);
  FR_SUB(bb, bb, t);
  FR_MUL(bb, bb, qc);
  FR_ADD(t, bb, e);
  FR_MUL(t, t, lk[4]);
  FR_ADD(out, sum, t);
}

/* -------------------------------------------------------------------- curve widgets */
/* JubJub twisted-Edwards d = -10240/10241 mod r, Montgomery */
static void edwards_d(uint64_t* out) {
  fr_t a, b;
  fr_small(a, 10240);
  fr_small(b, 10241);
  fr_inv(b, b);
  FR_MUL(a, a, b);
  fr_neg(out, a);
}
/* fixed-base scalar mul (dusk-plonk ecc/scalar_mul/fixed_base; zksnarks curve_scalar):
 * bit = d' - 2d; x_alpha = x_beta bit; y_alpha = bit^2 (y_beta - 1) + 1;
 * bit (bit-1)(bit+1) + (bit xy_beta - c) k + (x' (1 + c a b d_E) - (a y_alpha + b x_alpha)) k^2
 *   + (y' (1 - c a b d_E) - (b y_alpha + a x_alpha)) k^3    (a, b: point accumulator) */
static void fixed_base_terms(uint64_t* out, const uint64_t* ax, const uint64_t* axn,
                             const uint64_t* ay, const uint64_t* ayn, const uint64_t* xya,
                             const uint64_t* acc, const uint64_t* accn, const uint64_t* xb,
                             const uint64_t* yb, const uint64_t* xyb, fr_t* k,
                             const uint64_t* ed) {
  fr_t bit, t, u, bc, ya, xa, xy, prod, lhs, rhs, id, one;
  fr_set(one, FR_ONE);
  FR_ADD(t, acc, acc);
  FR_SUB(bit, accn, t);
  FR_SUB(t, bit, one);
  FR_MUL(bc, bit, t);
  FR_ADD(t, bit, one);
  FR_MUL(bc, bc, t);
  FR_MUL(t, bit, bit);
  FR_SUB(u, yb, one);
  FR_MUL(ya, t, u);
  FR_ADD(ya, ya, one);
  FR_MUL(xa, xb, bit);
  FR_MUL(xy, bit, xyb);
  FR_SUB(xy, xy, xya);
  FR_MUL(xy, xy, k[1]);
  FR_MUL(prod, xya, ax);
  FR_MUL(prod, prod, ay);
  FR_MUL(prod, prod, ed);
  fr_set(id, bc);
  FR_ADD(id, id, xy);
  FR_MUL(t, axn, prod); /* x check */
  FR_ADD(lhs, axn, t);
  FR_MUL(t, ax, ya);
  FR_MUL(u, ay, xa);
  FR_ADD(rhs, t, u);
  FR_SUB(t, lhs, rhs);
  FR_MUL(t, t, k[2]);
  FR_ADD(id, id, t);
  FR_MUL(t, ayn, prod); /* y check */
  FR_SUB(lhs, ayn, t);
  FR_MUL(t, ay, ya);
  FR_MUL(u, ax, xa);
  FR_ADD(rhs, t, u);
  FR_SUB(t, lhs, rhs);
  FR_MUL(t, t, k[3]);
  FR_ADD(out, id, t);
}
/* variable-base addition (dusk-plonk ecc/curve_addition; zksnarks curve_addtion):
 * (x1 y2 - x1y2') + (x1y2' + y1 x2 - x3 (1 + d_E x1y2' y1 x2)) k
 *                 + (y1 y2 + x1 x2 - y3 (1 - d_E x1y2' y1 x2)) k^2 */
static void var_base_terms(uint64_t* out, const uint64_t* x1, const uint64_t* x3,
                           const uint64_t* y1, const uint64_t* y3, const uint64_t* x2,
                           const uint64_t* y2, const uint64_t* x1y2, fr_t* k,
                           const uint64_t* ed) {
  fr_t xy, y1x2, y1y2, x1x2, dp, t, u, id;
  FR_MUL(xy, x1, y2);
  FR_SUB(xy, xy, x1y2);
  FR_MUL(y1x2, y1, x2);
  FR_MUL(y1y2, y1, y2);
  FR_MUL(x1x2, x1, x2);
  FR_MUL(dp, ed, x1y2);
  FR_MUL(dp, dp, y1x2);
  FR_ADD(t, x1y2, y1x2);
  FR_MUL(u, x3, dp);
  FR_ADD(u, u, x3);
  FR_SUB(t, t, u);
  FR_MUL(t, t, k[1]);
  FR_ADD(id, xy, t);
  FR_ADD(t, y1y2, x1x2);
  FR_MUL(u, y3, dp);
  FR_SUB(u, y3, u);
  FR_SUB(t, t, u);
  FR_MUL(t, t, k[2]);
  FR_ADD(out, id, t);
}

/* ------------------------------------------------------------------------- circuit */
/* selector order of plk_constraint / the composer */
enum { S_QM, S_QL, S_QR, S_QO, S_Q4, S_QC, S_QARITH, S_QRANGE, S_QLOGIC, S_QFIXED, S_QVAR, S_COUNT };

static uint32_t log2_ceil_u64(uint64_t v) {
  uint32_t k = 0;
  while ((1ull << k) < v) ++k;
  return k;
}

/* commit over the trimmed SRS prefix (trailing zeros stripped first) */
static int commit(const uint64_t* srs, size_t n_trim, const uint64_t* p, size_t len, uint64_t* out,
                  int threads, uint64_t* msm_ns) {
  while (len > 0 && fr_is_zero(p + 4 * (len - 1))) --len;
  if (len > n_trim) return ORC_E_DEGREE;
  const uint64_t t0 = now_ns();
  if (len == 0) {
    memset(out, 0, 13 * 8);
    out[12] = 1;
  } else if (orc_msm(srs, p, len, out, threads)) {
    return ORC_E_OOM;
  }
  if (msm_ns) *msm_ns += now_ns() - t0;
  return ORC_OK;
}

/* in-place transform of a zero-padded 2^log_n buffer, timed */
static void ntt_timed(uint64_t* data, uint32_t log_n, int dir, int coset, int threads, uint64_t* ns) {
  const uint64_t t0 = now_ns();
  orc_ntt(data, log_n, dir, coset, threads);
  if (ns) *ns += now_ns() - t0;
}

/*
 * Key compile + create_proof. Inputs: m gates in plk_constraint layout (11 Montgomery Fr
 * selectors, wires a,b,o,d, has_public, pad, public_input: 51 u64 words per gate), the
 * witness (Montgomery Fr), the SRS points (13-word ABI, >= next_pow2(m+6)+8 of them), the
 * transcript label, the blinding seed. If vk_in is non-null its 15 commitments are used
 * instead of committing the selectors and sigmas (the CPU-baseline timing mode).
 * Outputs: vk (15 x 13 words), proof commitments (11 x 13), evaluations (16 x 4 words,
 * plk_proof order), public inputs (count written to *pi_count, up to pi_cap values), and
 * timing[8] in ns: {key compile, proof MSMs, proof NTTs, quotient loop, grand product,
 * linearisation + openings, create_proof total, transcript}.
 */
int orc_prove(const uint64_t* gates, size_t m, const uint64_t* witness, size_t nw,
              const uint64_t* srs, size_t srs_len, const char* label, uint64_t seed,
              int threads, const uint64_t* vk_in, uint64_t* vk_out, uint64_t* proof_comms,
              uint64_t* proof_evals, uint64_t* pis_out, size_t pi_cap, size_t* pi_count,
              uint64_t* timing) {
  if (threads > 0) omp_set_num_threads(threads);
  uint64_t tm[8] = {0};
  const uint64_t t_start = now_ns();
  if (m == 0) return ORC_E_ARG;
  const uint32_t k = log2_ceil_u64(m);
  const uint64_t n = 1ull << k, n8 = 8 * n;
  const size_t n_trim = (size_t)(1ull << log2_ceil_u64(m + 6)) + 8;
  if (srs_len < n_trim || k + 3 > 30) return ORC_E_ARG;
  const size_t GW = 51; /* u64 words per plk_constraint: 11 selectors, 6 u32, public input */
  for (size_t i = 0; i < m; ++i) {
    const uint64_t* g = gates + GW * i;
    const uint32_t* w = (const uint32_t*)(g + 44);
    for (int c = 0; c < 4; ++c)
      if (w[c] >= nw) return ORC_E_ARG;
  }
  fr_t one, K[4];
  fr_set(one, FR_ONE);
  fr_set(K[0], FR_ONE);
  fr_from_u64(K[1], 7);
  fr_from_u64(K[2], 13);
  fr_from_u64(K[3], 17);

  /* =================================================================== key compile */
  /* selectors padded to n, idft (key.rs:89-131) */
  uint64_t* qc = fr_alloc(S_COUNT * n);
  for (size_t i = 0; i < m; ++i)
    for (int q = 0; q < S_COUNT; ++q) fr_set(qc + 4 * (q * n + i), gates + GW * i + 4 * q);
  for (int q = 0; q < S_COUNT; ++q) ntt_timed(qc + 4 * q * n, k, -1, 0, threads, &tm[2]);
  /* sigma (permutation.rs:108-141): each witness's wires in insertion order (gate order,
   * columns a, b, o, d), wire -> next, last -> first; identity for unused wires */
  uint64_t* wire_next = (uint64_t*)malloc(8 * 4 * n);
  uint64_t* head = (uint64_t*)malloc(8 * (nw ? nw : 1));
  uint64_t* tail = (uint64_t*)malloc(8 * (nw ? nw : 1));
  const uint64_t NONE = ~0ull;
  for (size_t j = 0; j < nw; ++j) head[j] = tail[j] = NONE;
  for (uint64_t wv = 0; wv < 4 * n; ++wv) wire_next[wv] = NONE;
  for (size_t i = 0; i < m; ++i) {
    const uint32_t* w = (const uint32_t*)(gates + GW * i + 44);
    for (int c = 0; c < 4; ++c) {
      const uint64_t wire = 4 * i + c; /* (gate i, column c) */
      if (tail[w[c]] == NONE)
        head[w[c]] = wire;
      else
        wire_next[tail[w[c]]] = wire;
      tail[w[c]] = wire;
    }
  }
  uint64_t* sigma_map = (uint64_t*)malloc(8 * 4 * n); /* [col][row] -> target wire */
  for (uint64_t i = 0; i < n; ++i)
    for (int c = 0; c < 4; ++c) sigma_map[c * n + i] = 4 * i + c;
  for (size_t j = 0; j < nw; ++j)
    for (uint64_t cur = head[j]; cur != NONE; cur = wire_next[cur]) {
      const uint64_t nx = wire_next[cur] == NONE ? head[j] : wire_next[cur];
      sigma_map[(cur & 3) * n + (cur >> 2)] = nx;
    }
  free(wire_next);
  free(head);
  free(tail);
  /* Lagrange encodings w^row * K_col (permutation.rs:143-168), then idft */
  uint64_t* elem = fr_alloc(n);
  orc_elements(k, elem, threads);
  uint64_t* sc = fr_alloc(4 * n);
  for (int c = 0; c < 4; ++c)
    for (uint64_t i = 0; i < n; ++i) {
      const uint64_t t = sigma_map[c * n + i];
      FR_MUL(sc + 4 * (c * n + i), elem + 4 * (t >> 2), K[t & 3]);
    }
  free(sigma_map);
  for (int c = 0; c < 4; ++c) ntt_timed(sc + 4 * c * n, k, -1, 0, threads, &tm[2]);
  /* verifier key commitments (key.rs:138-159), transcript order */
  static const int vk_sel[11] = {S_QM, S_QL, S_QR, S_QO, S_QC, S_Q4, S_QARITH, S_QRANGE,
                                 S_QLOGIC, S_QFIXED, S_QVAR};
  uint64_t vk[15 * 13];
  if (vk_in) {
    memcpy(vk, vk_in, sizeof vk);
  } else {
    for (int j = 0; j < 11; ++j)
      if (commit(srs, n_trim, qc + 4 * vk_sel[j] * n, n, vk + 13 * j, threads, &tm[1]) != ORC_OK) {
        memset(vk + 13 * j, 0, 13 * 8); /* unwrap_or_default: identity */
        vk[13 * j + 12] = 1;
      }
    for (int c = 0; c < 4; ++c) {
      const int st = commit(srs, n_trim, sc + 4 * c * n, n, vk + 13 * (11 + c), threads, &tm[1]);
      if (st != ORC_OK) return st;
    }
  }
  if (vk_out) memcpy(vk_out, vk, sizeof vk);
  /* 8n coset evaluations of selectors and sigmas (key.rs:220-245) */
  static const int sel8_src[11] = {S_QM, S_QL, S_QR, S_QO, S_Q4, S_QC, S_QARITH, S_QRANGE,
                                   S_QLOGIC, S_QFIXED, S_QVAR};
  uint64_t* sel8 = fr_alloc(11 * n8);
  uint64_t* sig8 = fr_alloc(4 * n8);
  for (int j = 0; j < 11; ++j) {
    memcpy(sel8 + 4 * j * n8, qc + 4 * sel8_src[j] * n, 32 * n);
    ntt_timed(sel8 + 4 * j * n8, k + 3, 1, 1, threads, &tm[2]);
  }
  for (int c = 0; c < 4; ++c) {
    memcpy(sig8 + 4 * c * n8, sc + 4 * c * n, 32 * n);
    ntt_timed(sig8 + 4 * c * n8, k + 3, 1, 1, threads, &tm[2]);
  }
  /* v_h over the 8n coset: (g w8^i)^n - 1 (key.rs:291) */
  uint64_t* vh = fr_alloc(n8);
  orc_vanishing(k + 3, n, vh);
  int has_range = 0, has_logic = 0, has_fixed = 0, has_var = 0;
  for (size_t i = 0; i < m; ++i) {
    has_range |= !fr_is_zero(gates + GW * i + 4 * S_QRANGE);
    has_logic |= !fr_is_zero(gates + GW * i + 4 * S_QLOGIC);
    has_fixed |= !fr_is_zero(gates + GW * i + 4 * S_QFIXED);
    has_var |= !fr_is_zero(gates + GW * i + 4 * S_QVAR);
  }
  tm[0] = now_ns() - t_start;

  /* ==================================================================== create_proof */
  const uint64_t t_prove = now_ns();
  uint64_t t_tr = 0, t0;
  tm[1] = tm[2] = 0; /* from here on the MSM / NTT timers cover create_proof only */
  orc_rng rng = {seed};
  orc_transcript tr;
  t0 = now_ns();
  tr_init(&tr, (const uint8_t*)label, strlen(label));
  tr_append_message(&tr, "dom-sep", (const uint8_t*)"circuit_size", 12);
  tr_append_u64(&tr, "n", m);
  static const char* vk_labels[15] = {"q_m", "q_l", "q_r", "q_o", "q_c", "q_4", "q_arith",
                                      "q_range", "q_logic", "q_fixed_group_add",
                                      "q_variable_group_add", "s_sigma_1", "s_sigma_2",
                                      "s_sigma_3", "s_sigma_4"};
  for (int j = 0; j < 15; ++j) tr_append_commitment(&tr, vk_labels[j], vk + 13 * j);
  /* public inputs: Plonk::instance, sorted by gate index (prover.rs:90-105) */
  uint64_t* pil = fr_alloc(n);
  size_t npi = 0;
  for (size_t i = 0; i < m; ++i) {
    const uint64_t* g = gates + GW * i;
    const uint32_t has_pi = ((const uint32_t*)(g + 44))[4];
    if (!has_pi) continue;
    tr_append_scalar(&tr, "pi", g + 47);
    fr_set(pil + 4 * i, g + 47);
    if (pis_out && npi < pi_cap) fr_set(pis_out + 4 * npi, g + 47);
    ++npi;
  }
  if (pi_count) *pi_count = npi;
  t_tr += now_ns() - t0;

  /* ---- round 1: wires (prover.rs:107-158) */
  const size_t S = n + 8; /* padded stride: blinded wires have n + 2 coefficients */
  uint64_t* wl = fr_alloc(4 * n); /* Lagrange values, kept for the grand product */
  uint64_t* wc = fr_alloc(4 * S);
  for (size_t i = 0; i < m; ++i) {
    const uint32_t* w = (const uint32_t*)(gates + GW * i + 44);
    for (int c = 0; c < 4; ++c) fr_set(wl + 4 * (c * n + i), witness + 4 * w[c]);
  }
  for (int c = 0; c < 4; ++c) {
    uint64_t* p = wc + 4 * c * S;
    memcpy(p, wl + 4 * c * n, 32 * n);
    ntt_timed(p, k, -1, 0, threads, &tm[2]);
    /* blind(1): + (b0 + b1 X)(X^n - 1) */
    for (int j = 0; j < 2; ++j) {
      fr_t b;
      rng_fr(&rng, b);
      FR_SUB(p + 4 * j, p + 4 * j, b);
      FR_ADD(p + 4 * (n + j), p + 4 * (n + j), b);
    }
  }
  uint64_t wcom[4][13];
  for (int c = 0; c < 4; ++c) {
    const int st = commit(srs, n_trim, wc + 4 * c * S, n + 2, wcom[c], threads, &tm[1]);
    if (st != ORC_OK) return st;
  }
  t0 = now_ns();
  tr_append_commitment(&tr, "a_w", wcom[0]);
  tr_append_commitment(&tr, "b_w", wcom[1]);
  tr_append_commitment(&tr, "c_w", wcom[2]);
  tr_append_commitment(&tr, "d_w", wcom[3]);
  fr_t beta, gamma;
  tr_challenge_scalar(&tr, "beta", beta);
  tr_append_scalar(&tr, "beta", beta);
  tr_challenge_scalar(&tr, "gamma", gamma);
  t_tr += now_ns() - t0;

  /* ---- round 2: grand product (permutation.rs:205-300) */
  uint64_t* zc = fr_alloc(S);
  {
    const uint64_t tg = now_ns(), ntt_before = tm[2];
    uint64_t* sig_lag = fr_alloc(4 * n); /* fft.dft of each sigma polynomial */
    memcpy(sig_lag, sc, 32 * 4 * n);
    for (int c = 0; c < 4; ++c) ntt_timed(sig_lag + 4 * c * n, k, 1, 0, threads, &tm[2]);
    uint64_t* prod = fr_alloc(n);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)n; ++i) {
      fr_t nu, de, t, u;
      fr_set(nu, FR_ONE);
      fr_set(de, FR_ONE);
      for (int c = 0; c < 4; ++c) {
        const uint64_t* w = wl + 4 * (c * n + i);
        FR_MUL(t, beta, K[c]);
        FR_MUL(t, t, elem + 4 * i);
        FR_ADD(t, t, w);
        FR_ADD(t, t, gamma);
        FR_MUL(nu, nu, t);
        FR_MUL(u, beta, sig_lag + 4 * (c * n + i));
        FR_ADD(u, u, w);
        FR_ADD(u, u, gamma);
        FR_MUL(de, de, u);
      }
      fr_inv(de, de); /* one inversion per gate, as the reference's map */
      FR_MUL(prod + 4 * i, nu, de);
    }
    fr_t state;
    fr_set(state, FR_ONE);
    for (uint64_t i = 0; i < n; ++i) { /* z_0 = 1, z_{i+1} = z_i prod_i, last dropped */
      fr_set(zc + 4 * i, state);
      FR_MUL(state, state, prod + 4 * i);
    }
    free(prod);
    free(sig_lag);
    tm[4] += (now_ns() - tg) - (tm[2] - ntt_before);
    ntt_timed(zc, k, -1, 0, threads, &tm[2]);
    for (int j = 0; j < 3; ++j) { /* blind(2) */
      fr_t b;
      rng_fr(&rng, b);
      FR_SUB(zc + 4 * j, zc + 4 * j, b);
      FR_ADD(zc + 4 * (n + j), zc + 4 * (n + j), b);
    }
  }
  uint64_t zcom[13];
  {
    const int st = commit(srs, n_trim, zc, n + 3, zcom, threads, &tm[1]);
    if (st != ORC_OK) return st;
  }
  t0 = now_ns();
  tr_append_commitment(&tr, "z", zcom);
  fr_t alpha, range_sep, logic_sep, fixed_sep, var_sep;
  tr_challenge_scalar(&tr, "alpha", alpha);
  tr_challenge_scalar(&tr, "range separation challenge", range_sep);
  tr_challenge_scalar(&tr, "logic separation challenge", logic_sep);
  tr_challenge_scalar(&tr, "fixed base separation challenge", fixed_sep);
  tr_challenge_scalar(&tr, "variable base separation challenge", var_sep);
  t_tr += now_ns() - t0;

  /* ---- round 3: quotient (quotient_poly.rs) */
  ntt_timed(pil, k, -1, 0, threads, &tm[2]); /* pi_poly = idft(dense public inputs) */
  uint64_t* ev[5]; /* z, a, b, c, d over the 8n coset, + 8 wrap-around rows */
  for (int j = 0; j < 5; ++j) {
    ev[j] = fr_alloc(n8 + 8);
    const uint64_t* src = j == 0 ? zc : wc + 4 * (j - 1) * S;
    memcpy(ev[j], src, 32 * (j == 0 ? n + 3 : n + 2));
    ntt_timed(ev[j], k + 3, 1, 1, threads, &tm[2]);
    memcpy(ev[j] + 4 * n8, ev[j], 32 * 8);
  }
  uint64_t* pi8 = fr_alloc(n8);
  memcpy(pi8, pil, 32 * n);
  ntt_timed(pi8, k + 3, 1, 1, threads, &tm[2]);
  uint64_t* l18 = fr_alloc(n8); /* L1 * alpha^2: idft_n(alpha^2 e_0), then 8n coset dft */
  fr_t alpha2;
  FR_MUL(alpha2, alpha, alpha);
  fr_set(l18, alpha2);
  ntt_timed(l18, k, -1, 0, threads, &tm[2]);
  ntt_timed(l18, k + 3, 1, 1, threads, &tm[2]);
  fr_t kappa, kappa2, kappa3, lk[5];
  FR_MUL(kappa, range_sep, range_sep);
  FR_MUL(kappa2, kappa, kappa);
  FR_MUL(kappa3, kappa2, kappa);
  fr_set(lk[0], FR_ONE); /* logic: 1, k, k^2, k^3, k^4 with k = logic_sep^2 */
  FR_MUL(lk[1], logic_sep, logic_sep);
  for (int j = 2; j < 5; ++j) FR_MUL(lk[j], lk[j - 1], lk[1]);
  fr_t fk[4], vbk[3], ed;
  fr_set(fk[0], FR_ONE); /* fixed base: 1, k, k^2, k^3 with k = sep^2 */
  FR_MUL(fk[1], fixed_sep, fixed_sep);
  FR_MUL(fk[2], fk[1], fk[1]);
  FR_MUL(fk[3], fk[2], fk[1]);
  fr_set(vbk[0], FR_ONE); /* variable base: 1, k, k^2 */
  FR_MUL(vbk[1], var_sep, var_sep);
  FR_MUL(vbk[2], vbk[1], vbk[1]);
  edwards_d(ed);
  uint64_t* quot = fr_alloc(n8);
  {
    const uint64_t tq = now_ns();
    uint64_t* t1 = fr_alloc(n8);
    /* compute_circuit_satisfiability_equation: sequential loop (quotient_poly.rs:152) */
    fr_t two, three, four;
    FR_ADD(two, one, one);
    FR_ADD(three, two, one);
    FR_ADD(four, two, two);
    for (uint64_t i = 0; i < n8; ++i) {
      const uint64_t *a = ev[1] + 4 * i, *b = ev[2] + 4 * i, *c = ev[3] + 4 * i, *d = ev[4] + 4 * i;
      fr_t acc, t;
      /* arithmetic: q_arith (q_m a b + q_l a + q_r b + q_o c + q_4 d + q_c) */
      FR_MUL(t, a, b);
      FR_MUL(acc, sel8 + 4 * (0 * n8 + i), t);
      FR_MUL(t, sel8 + 4 * (1 * n8 + i), a);
      FR_ADD(acc, acc, t);
      FR_MUL(t, sel8 + 4 * (2 * n8 + i), b);
      FR_ADD(acc, acc, t);
      FR_MUL(t, sel8 + 4 * (3 * n8 + i), c);
      FR_ADD(acc, acc, t);
      FR_MUL(t, sel8 + 4 * (4 * n8 + i), d);
      FR_ADD(acc, acc, t);
      FR_ADD(acc, acc, sel8 + 4 * (5 * n8 + i));
      FR_MUL(acc, acc, sel8 + 4 * (6 * n8 + i));
      FR_ADD(acc, acc, pi8 + 4 * i);
      /* range: sep q_range (D(c-4d) + D(b-4c) k + D(a-4b) k^2 + D(d_next-4a) k^3) */
      if (has_range) {
        const uint64_t* dn = ev[4] + 4 * (i + 8);
        const uint64_t* pairs[4][2] = {{c, d}, {b, c}, {a, b}, {dn, a}};
        const uint64_t* ks[4] = {one, kappa, kappa2, kappa3};
        fr_t sum;
        fr_zero(sum);
        for (int q = 0; q < 4; ++q) {
          fr_t f, f1, f2, f3, dl;
          FR_MUL(f, four, pairs[q][1]);
          FR_SUB(f, pairs[q][0], f);
          FR_SUB(f1, f, one);
          FR_SUB(f2, f, two);
          FR_SUB(f3, f, three);
          FR_MUL(dl, f, f1);
          FR_MUL(f2, f2, f3);
          FR_MUL(dl, dl, f2);
          FR_MUL(dl, dl, ks[q]);
          FR_ADD(sum, sum, dl);
        }
        FR_MUL(sum, sum, sel8 + 4 * (7 * n8 + i));
        FR_MUL(sum, sum, range_sep);
        FR_ADD(acc, acc, sum);
      }
      /* logic: sep q_logic (D(a') + D(b') k + D(d') k^2 + (c - a'b') k^3 + xor_and k^4) */
      if (has_logic) {
        const uint64_t* an = ev[1] + 4 * (i + 8);
        const uint64_t* bn = ev[2] + 4 * (i + 8);
        const uint64_t* dn = ev[4] + 4 * (i + 8);
        fr_t sum;
        logic_terms(sum, a, an, b, bn, c, d, dn, sel8 + 4 * (5 * n8 + i), lk);
        FR_MUL(sum, sum, sel8 + 4 * (8 * n8 + i));
        FR_MUL(sum, sum, logic_sep);
        FR_ADD(acc, acc, sum);
      }
      if (has_fixed) {
        fr_t w;
        fixed_base_terms(w, a, ev[1] + 4 * (i + 8), b, ev[2] + 4 * (i + 8), c, d, ev[4] + 4 * (i + 8),
                         sel8 + 4 * (1 * n8 + i), sel8 + 4 * (2 * n8 + i), sel8 + 4 * (5 * n8 + i),
                         fk, ed);
        FR_MUL(w, w, sel8 + 4 * (9 * n8 + i));
        FR_MUL(w, w, fixed_sep);
        FR_ADD(acc, acc, w);
      }
      if (has_var) {
        fr_t w;
        var_base_terms(w, a, ev[1] + 4 * (i + 8), b, ev[2] + 4 * (i + 8), c, d, ev[4] + 4 * (i + 8),
                       vbk, ed);
        FR_MUL(w, w, sel8 + 4 * (10 * n8 + i));
        FR_MUL(w, w, var_sep);
        FR_ADD(acc, acc, w);
      }
      fr_set(t1 + 4 * i, acc);
    }
    /* compute_permutation_checks: parallel loop (quotient_poly.rs:238-262) */
    uint64_t* el8 = fr_alloc(n8);
    orc_elements(k + 3, el8, threads);
    fr_t g;
    fr_from_u64(g, 7);
#pragma omp parallel for schedule(static)
    for (int64_t ii = 0; ii < (int64_t)n8; ++ii) {
      const uint64_t i = (uint64_t)ii;
      fr_t x, bx, idt, cp, t, u;
      FR_MUL(x, g, el8 + 4 * i);
      FR_MUL(bx, beta, x);
      fr_set(idt, ev[0] + 4 * i); /* z_i */
      FR_MUL(idt, idt, alpha);
      fr_set(cp, ev[0] + 4 * (i + 8)); /* z_next */
      FR_MUL(cp, cp, alpha);
      for (int c = 0; c < 4; ++c) {
        const uint64_t* w = ev[1 + c] + 4 * i;
        FR_MUL(t, K[c], bx);
        FR_ADD(t, t, w);
        FR_ADD(t, t, gamma);
        FR_MUL(idt, idt, t);
        FR_MUL(u, beta, sig8 + 4 * (c * n8 + i));
        FR_ADD(u, u, w);
        FR_ADD(u, u, gamma);
        FR_MUL(cp, cp, u);
      }
      FR_SUB(t, ev[0] + 4 * i, one); /* (z - 1) L1 alpha^2 */
      FR_MUL(t, t, l18 + 4 * i);
      FR_SUB(idt, idt, cp);
      FR_ADD(quot + 4 * i, idt, t);
    }
    free(el8);
    /* quotient: (t1 + t2) / v_h, one inversion per point in a sequential loop (:99-107) */
    for (uint64_t i = 0; i < n8; ++i) {
      fr_t num, inv;
      FR_ADD(num, t1 + 4 * i, quot + 4 * i);
      fr_inv(inv, vh + 4 * i);
      FR_MUL(quot + 4 * i, num, inv);
    }
    free(t1);
    tm[3] += now_ns() - tq;
  }
  ntt_timed(quot, k + 3, -1, 1, threads, &tm[2]); /* t(X), 8n coefficients */
  const uint64_t* tc = quot;
  uint64_t tcom[4][13];
  for (int j = 0; j < 4; ++j) {
    const int st = commit(srs, n_trim, tc + 4 * j * n, j < 3 ? n : 5 * n, tcom[j], threads, &tm[1]);
    if (st != ORC_OK) return st;
  }
  t0 = now_ns();
  tr_append_commitment(&tr, "t_low", tcom[0]);
  tr_append_commitment(&tr, "t_mid", tcom[1]);
  tr_append_commitment(&tr, "t_high", tcom[2]);
  tr_append_commitment(&tr, "t_4", tcom[3]);
  fr_t zeta, zw, w_n;
  tr_challenge_scalar(&tr, "z_challenge", zeta);
  t_tr += now_ns() - t0;
  orc_fr_omega(k, w_n);
  FR_MUL(zw, zeta, w_n);

  /* ---- round 4/5: evaluations and linearisation (linearization_poly.rs:52-134) */
  const uint64_t tl = now_ns();
  fr_t t_e, a_e, b_e, c_e, d_e, s1_e, s2_e, s3_e, qar_e, qc_e, ql_e, qr_e, an_e, bn_e, dn_e, perm_e;
  poly_eval(t_e, tc, n8, zeta);
  poly_eval(a_e, wc + 0 * 4 * S, n + 2, zeta);
  poly_eval(b_e, wc + 1 * 4 * S, n + 2, zeta);
  poly_eval(c_e, wc + 2 * 4 * S, n + 2, zeta);
  poly_eval(d_e, wc + 3 * 4 * S, n + 2, zeta);
  poly_eval(s1_e, sc + 0 * 4 * n, n, zeta);
  poly_eval(s2_e, sc + 1 * 4 * n, n, zeta);
  poly_eval(s3_e, sc + 2 * 4 * n, n, zeta);
  poly_eval(qar_e, qc + 4 * S_QARITH * n, n, zeta);
  poly_eval(qc_e, qc + 4 * S_QC * n, n, zeta);
  poly_eval(ql_e, qc + 4 * S_QL * n, n, zeta);
  poly_eval(qr_e, qc + 4 * S_QR * n, n, zeta);
  poly_eval(an_e, wc + 0 * 4 * S, n + 2, zw);
  poly_eval(bn_e, wc + 1 * 4 * S, n + 2, zw);
  poly_eval(dn_e, wc + 3 * 4 * S, n + 2, zw);
  poly_eval(perm_e, zc, n + 3, zw);
  /* r(X) = arithmetic::linearize + range::linearize + permutation::linearize */
  uint64_t* rc = fr_alloc(n + 3);
  {
    fr_t s, t;
    FR_MUL(t, a_e, b_e);
    FR_MUL(s, qar_e, t);
    poly_axpy(rc, qc + 4 * S_QM * n, n, s);
    FR_MUL(s, qar_e, a_e);
    poly_axpy(rc, qc + 4 * S_QL * n, n, s);
    FR_MUL(s, qar_e, b_e);
    poly_axpy(rc, qc + 4 * S_QR * n, n, s);
    FR_MUL(s, qar_e, c_e);
    poly_axpy(rc, qc + 4 * S_QO * n, n, s);
    FR_MUL(s, qar_e, d_e);
    poly_axpy(rc, qc + 4 * S_Q4 * n, n, s);
    poly_axpy(rc, qc + 4 * S_QC * n, n, qar_e);
    if (has_range) {
      fr_t two, three, four, sum;
      FR_ADD(two, one, one);
      FR_ADD(three, two, one);
      FR_ADD(four, two, two);
      const uint64_t* pairs[4][2] = {{c_e, d_e}, {b_e, c_e}, {a_e, b_e}, {dn_e, a_e}};
      const uint64_t* ks[4] = {one, kappa, kappa2, kappa3};
      fr_zero(sum);
      for (int q = 0; q < 4; ++q) {
        fr_t f, f1, f2, f3, dl;
        FR_MUL(f, four, pairs[q][1]);
        FR_SUB(f, pairs[q][0], f);
        FR_SUB(f1, f, one);
        FR_SUB(f2, f, two);
        FR_SUB(f3, f, three);
        FR_MUL(dl, f, f1);
        FR_MUL(f2, f2, f3);
        FR_MUL(dl, dl, f2);
        FR_MUL(dl, dl, ks[q]);
        FR_ADD(sum, sum, dl);
      }
      FR_MUL(sum, sum, range_sep);
      poly_axpy(rc, qc + 4 * S_QRANGE * n, n, sum);
    }
    if (has_logic) {
      fr_t sum;
      logic_terms(sum, a_e, an_e, b_e, bn_e, c_e, d_e, dn_e, qc_e, lk);
      FR_MUL(sum, sum, logic_sep);
      poly_axpy(rc, qc + 4 * S_QLOGIC * n, n, sum);
    }
    if (has_fixed) {
      fr_t w;
      fixed_base_terms(w, a_e, an_e, b_e, bn_e, c_e, d_e, dn_e, ql_e, qr_e, qc_e, fk, ed);
      FR_MUL(w, w, fixed_sep);
      poly_axpy(rc, qc + 4 * S_QFIXED * n, n, w);
    }
    if (has_var) {
      fr_t w;
      var_base_terms(w, a_e, an_e, b_e, bn_e, c_e, d_e, dn_e, vbk, ed);
      FR_MUL(w, w, var_sep);
      poly_axpy(rc, qc + 4 * S_QVAR * n, n, w);
    }
    /* identity: z(X) (a + b z + g)(b + b K1 z + g)(c + b K2 z + g)(d + b K3 z + g) alpha */
    fr_t bz, idc;
    FR_MUL(bz, beta, zeta);
    fr_set(idc, alpha);
    const uint64_t* ws[4] = {a_e, b_e, c_e, d_e};
    for (int c = 0; c < 4; ++c) {
      FR_MUL(t, K[c], bz);
      FR_ADD(t, t, ws[c]);
      FR_ADD(t, t, gamma);
      FR_MUL(idc, idc, t);
    }
    poly_axpy(rc, zc, n + 3, idc);
    /* copy: -sigma_4(X) (a + b s1 + g)(b + b s2 + g)(c + b s3 + g) beta perm_eval alpha */
    fr_t cpc;
    const uint64_t* ss[3] = {s1_e, s2_e, s3_e};
    FR_MUL(cpc, beta, perm_e);
    FR_MUL(cpc, cpc, alpha);
    for (int c = 0; c < 3; ++c) {
      FR_MUL(t, beta, ss[c]);
      FR_ADD(t, t, ws[c]);
      FR_ADD(t, t, gamma);
      FR_MUL(cpc, cpc, t);
    }
    fr_neg(cpc, cpc);
    poly_axpy(rc, sc + 4 * 3 * n, n, cpc);
    /* check_is_one: z(X) L1(z) alpha^2, L1(z) = (z^n - 1) / (n (z - 1)) */
    fr_t zh, l1, nn, dz;
    fr_pow_u64(zh, zeta, n);
    FR_SUB(zh, zh, one);
    fr_from_u64(nn, n);
    FR_SUB(dz, zeta, one);
    FR_MUL(nn, nn, dz);
    fr_inv(nn, nn);
    FR_MUL(l1, zh, nn);
    FR_MUL(l1, l1, alpha2);
    poly_axpy(rc, zc, n + 3, l1);
  }
  fr_t r_e;
  poly_eval(r_e, rc, n + 3, zeta);
  tm[5] += now_ns() - tl;
  t0 = now_ns();
  const char* elabels[17] = {"a_eval", "b_eval", "c_eval", "d_eval", "a_next_eval",
                             "b_next_eval", "d_next_eval", "s_sigma_1_eval", "s_sigma_2_eval",
                             "s_sigma_3_eval", "q_arith_eval", "q_c_eval", "q_l_eval",
                             "q_r_eval", "perm_eval", "t_eval", "r_eval"};
  const uint64_t* e17[17] = {a_e, b_e, c_e, d_e, an_e, bn_e, dn_e, s1_e, s2_e, s3_e,
                             qar_e, qc_e, ql_e, qr_e, perm_e, t_e, r_e};
  for (int i = 0; i < 17; ++i) tr_append_scalar(&tr, elabels[i], e17[i]);
  fr_t v1, v2;
  tr_challenge_scalar(&tr, "v_challenge", v1);
  tr_challenge_scalar(&tr, "v_challenge", v2);
  t_tr += now_ns() - t0;

  /* ---- openings (prover.rs:407-452, compute_aggregate_witness = sum v^i p_i, ruffini) */
  const uint64_t to = now_ns();
  fr_t zn, z2n, z3n, vp;
  fr_pow_u64(zn, zeta, n);
  FR_MUL(z2n, zn, zn);
  FR_MUL(z3n, z2n, zn);
  uint64_t* agg = fr_alloc(5 * n);
  poly_axpy(agg, tc, n, one); /* quot = t_low + z^n t_mid + z^2n t_high + z^3n t_4 */
  poly_axpy(agg, tc + 4 * n, n, zn);
  poly_axpy(agg, tc + 4 * 2 * n, n, z2n);
  poly_axpy(agg, tc + 4 * 3 * n, 5 * n, z3n);
  fr_set(vp, v1);
  poly_axpy(agg, rc, n + 3, vp);
  for (int c = 0; c < 4; ++c) {
    FR_MUL(vp, vp, v1);
    poly_axpy(agg, wc + 4 * c * S, n + 2, vp);
  }
  for (int c = 0; c < 3; ++c) {
    FR_MUL(vp, vp, v1);
    poly_axpy(agg, sc + 4 * c * n, n, vp);
  }
  uint64_t* w1 = fr_alloc(5 * n);
  poly_ruffini(w1, agg, 5 * n, zeta);
  uint64_t* agg2 = fr_alloc(n + 3);
  poly_axpy(agg2, zc, n + 3, one);
  fr_set(vp, v2);
  poly_axpy(agg2, wc + 4 * 0 * S, n + 2, vp);
  FR_MUL(vp, vp, v2);
  poly_axpy(agg2, wc + 4 * 1 * S, n + 2, vp);
  FR_MUL(vp, vp, v2);
  poly_axpy(agg2, wc + 4 * 3 * S, n + 2, vp);
  uint64_t* w2 = fr_alloc(n + 3);
  poly_ruffini(w2, agg2, n + 3, zw);
  tm[5] += now_ns() - to;
  uint64_t wcm[2][13];
  {
    int st = commit(srs, n_trim, w1, 5 * n - 1, wcm[0], threads, &tm[1]);
    if (st == ORC_OK) st = commit(srs, n_trim, w2, n + 2, wcm[1], threads, &tm[1]);
    if (st != ORC_OK) return st;
  }

  /* ---- proof (proof.rs:36-66), evaluations in plk_proof order */
  const uint64_t* comms[11] = {wcom[0], wcom[1], wcom[2], wcom[3], zcom, tcom[0],
                               tcom[1], tcom[2], tcom[3], wcm[0], wcm[1]};
  for (int j = 0; j < 11; ++j) memcpy(proof_comms + 13 * j, comms[j], 13 * 8);
  const uint64_t* evs[16] = {a_e, b_e, c_e, d_e, an_e, bn_e, dn_e, qar_e,
                             qc_e, ql_e, qr_e, s1_e, s2_e, s3_e, r_e, perm_e};
  for (int j = 0; j < 16; ++j) fr_set(proof_evals + 4 * j, evs[j]);
  tm[6] = now_ns() - t_prove;
  tm[7] = t_tr;
  if (timing) memcpy(timing, tm, sizeof tm);

  free(qc);
  free(sc);
  free(elem);
  free(sel8);
  free(sig8);
  free(vh);
  free(pil);
  free(wl);
  free(wc);
  free(zc);
  for (int j = 0; j < 5; ++j) free(ev[j]);
  free(pi8);
  free(l18);
  free(quot);
  free(rc);
  free(agg);
  free(w1);
  free(agg2);
  free(w2);
  return ORC_OK;
}
