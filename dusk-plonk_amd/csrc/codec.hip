// codec.hip — the Proof wire format (include/plk.h plk_proof_encode / plk_proof_decode).
//
// The reference derives parity-scale-codec Encode / Decode for Proof
// (/root/reference/src/prover/proof.rs:11,36): a SCALE struct is its fields' encodings
// concatenated in declaration order, with no framing — here 11 Commitment<G1Affine>
// (proof.rs:39-64) followed by ProofEvaluations (proof.rs:66). The element encodings belong to
// the un-vendored bls-12-381 / zksnarks crates and are ASSUMED (parity unpinned):
// a Commitment is its G1Affine, encoded field by field as x, y (Fq = [u64; 6], Montgomery
// limbs, each u64 little-endian) and is_infinity (bool: one byte 0/1) = 97 bytes; an Fr
// is [u64; 4] Montgomery limbs, little-endian = 32 bytes; ProofEvaluations in the order the
// prover builds it (linearization_poly.rs:117-134), the order of plk_proof. SCALE's Decode
// of a bool rejects bytes other than 0 and 1; this decoder also rejects limbs that are not
// canonical and finite points off y^2 = x^3 + 4 (the curve check the verifier relies on).
// The identity is encoded (x = 0, y = 0, is_infinity = 1); decode accepts that and the
// zkcrypto form (x = 0, y = one, is_infinity = 1) and rejects other coordinates under the flag.
// Host code only.
#include <cstring>

#include "internal.hpp"

using namespace plk;

namespace {

constexpr size_t kG1Bytes = 97, kFrBytes = 32, kComms = 11, kEvals = 16;
static_assert(PLK_PROOF_SCALE_BYTES == kComms * kG1Bytes + kEvals * kFrBytes, "layout");

void put_u64(uint8_t* p, uint64_t v) {
  for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (8 * i));
}
uint64_t get_u64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 0; i < 8; ++i) v |= (uint64_t)p[i] << (8 * i);
  return v;
}

// limbs (LE u64) < modulus (LE u32 words)
template <class C>
bool canonical(const uint64_t* l) {
  for (int i = C::N - 1; i >= 0; --i) {
    const uint32_t w = (uint32_t)(l[i / 2] >> (32 * (i % 2)));
    if (w != C::P[i]) return w < C::P[i];
  }
  return false;  // equal to the modulus
}

bool is_zero6(const uint64_t* l) {
  for (int i = 0; i < 6; ++i)
    if (l[i]) return false;
  return true;
}
// Montgomery one of Fp (R mod p), as LE u64 limbs
bool is_fp_one(const uint64_t* l) {
  const Fp one = fe_one<FpCfg>();
  for (int i = 0; i < 6; ++i)
    if (l[i] != ((uint64_t)one.v[2 * i] | ((uint64_t)one.v[2 * i + 1] << 32))) return false;
  return true;
}

template <class C>
Fe<C> fe_of(const uint64_t* l) {
  Fe<C> r;
  for (int i = 0; i < C::N; ++i) r.v[i] = (uint32_t)(l[i / 2] >> (32 * (i % 2)));
  return r;
}

bool on_curve(const plk_g1& g) {
  const Fp x = fe_of<FpCfg>(g.x), y = fe_of<FpCfg>(g.y);
  Fp four = fe_zero<FpCfg>();
  four.v[0] = 4;
  four = fe_to_mont(four);
  return fe_eq(fe_sqr(y), fe_add(fe_mul(fe_sqr(x), x), four));
}

// field order of proof.rs:39-66 / plk_proof
plk_g1 plk_proof::* const kCommField[kComms] = {
    &plk_proof::a_comm,     &plk_proof::b_comm,     &plk_proof::c_comm,
    &plk_proof::d_comm,     &plk_proof::z_comm,     &plk_proof::t_low_comm,
    &plk_proof::t_mid_comm, &plk_proof::t_high_comm, &plk_proof::t_4_comm,
    &plk_proof::w_z_chall_comm, &plk_proof::w_z_chall_w_comm};
plk_fr plk_proof::* const kEvalField[kEvals] = {
    &plk_proof::a_eval,         &plk_proof::b_eval,         &plk_proof::c_eval,
    &plk_proof::d_eval,         &plk_proof::a_next_eval,    &plk_proof::b_next_eval,
    &plk_proof::d_next_eval,    &plk_proof::q_arith_eval,   &plk_proof::q_c_eval,
    &plk_proof::q_l_eval,       &plk_proof::q_r_eval,       &plk_proof::s_sigma_1_eval,
    &plk_proof::s_sigma_2_eval, &plk_proof::s_sigma_3_eval, &plk_proof::r_poly_eval,
    &plk_proof::perm_eval};
const plk_g1* comm(const plk_proof* p, size_t i) { return &(p->*kCommField[i]); }
plk_g1* comm(plk_proof* p, size_t i) { return &(p->*kCommField[i]); }
const plk_fr* eval(const plk_proof* p, size_t i) { return &(p->*kEvalField[i]); }
plk_fr* eval(plk_proof* p, size_t i) { return &(p->*kEvalField[i]); }

}  // namespace

extern "C" {

int plk_proof_encode(const plk_proof* proof, uint8_t* out, size_t cap, size_t* len) {
  if (!proof) return PLK_E_ARG;
  if (len) *len = PLK_PROOF_SCALE_BYTES;
  if (!out) return PLK_OK;  // size query
  if (cap < PLK_PROOF_SCALE_BYTES) return PLK_E_ARG;
  uint8_t* o = out;
  for (size_t i = 0; i < kComms; ++i) {
    const plk_g1* g = comm(proof, i);
    for (int k = 0; k < 6; ++k) put_u64(o + 8 * k, g->x[k]);
    for (int k = 0; k < 6; ++k) put_u64(o + 48 + 8 * k, g->y[k]);
    o[96] = g->infinity ? 1 : 0;
    o += kG1Bytes;
  }
  for (size_t i = 0; i < kEvals; ++i) {
    const plk_fr* f = eval(proof, i);
    for (int k = 0; k < 4; ++k) put_u64(o + 8 * k, f->l[k]);
    o += kFrBytes;
  }
  return PLK_OK;
}

int plk_proof_decode(const uint8_t* in, size_t len, plk_proof* proof) {
  if (!in || !proof || len != PLK_PROOF_SCALE_BYTES) return PLK_E_ARG;
  plk_proof p;
  std::memset(&p, 0, sizeof p);
  const uint8_t* q = in;
  for (size_t i = 0; i < kComms; ++i) {
    plk_g1* g = comm(&p, i);
    for (int k = 0; k < 6; ++k) g->x[k] = get_u64(q + 8 * k);
    for (int k = 0; k < 6; ++k) g->y[k] = get_u64(q + 48 + 8 * k);
    if (q[96] > 1) return PLK_E_ARG;
    g->infinity = q[96];
    if (!canonical<FpCfg>(g->x) || !canonical<FpCfg>(g->y)) return PLK_E_ARG;
    if (g->infinity) {
      // the identity's two known encodings: (0, 0, true) (this encoder) and (0, one, true)
      // (zkcrypto-style crates); any other coordinates under the flag are rejected, so
      // decode stays injective up to these two. Normalised to this ABI's (0, 0, 1).
      if (!is_zero6(g->x) || !(is_zero6(g->y) || is_fp_one(g->y))) return PLK_E_ARG;
      std::memset(g->x, 0, sizeof g->x);
      std::memset(g->y, 0, sizeof g->y);
    } else if (!on_curve(*g)) {
      return PLK_E_ARG;
    }
    q += kG1Bytes;
  }
  for (size_t i = 0; i < kEvals; ++i) {
    plk_fr* f = eval(&p, i);
    for (int k = 0; k < 4; ++k) f->l[k] = get_u64(q + 8 * k);
    if (!canonical<FrCfg>(f->l)) return PLK_E_ARG;
    q += kFrBytes;
  }
  *proof = p;
  return PLK_OK;
}

}  // extern "C"
