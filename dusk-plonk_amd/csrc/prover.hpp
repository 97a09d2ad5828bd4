// prover.hpp — composer, proving key and prover objects behind the plk_composer / plk_key /
// plk_prove entry points of include/plk.h, and the kernel-argument structs of
// prover_kernels.hip.
#pragma once
#include <map>
#include <string>
#include <vector>

#include "internal.hpp"

namespace plk {

// ---- kernel arguments --------------------------------------------------------------
struct BlindArgs {
  Fr r[4];
  uint32_t count;
};
// PI(X) of a few public inputs straight from its definition (pk_pi_coef)
constexpr int kPiDirect = 16;
struct PiDirect {
  uint64_t idx[kPiDirect];  // gate index of each public input
  Fr c[kPiDirect];          // its value times n^-1 (R domain)
  uint32_t count;
};
// the blinding of up to 4 polynomials in one launch (round 1's four wires)
struct BlindBatch {
  Fr* poly[4];
  BlindArgs b[4];
  uint32_t npoly;
};

// selector rows of the quotient-domain evaluation table
enum { SEL_QM = 0, SEL_QL, SEL_QR, SEL_QO, SEL_Q4, SEL_QC, SEL_QARITH, SEL_QRANGE, SEL_QLOGIC,
       SEL_QFIXED, SEL_QVAR, SEL_COUNTQ };

// The quotient domain (round 3). The reference evaluates the quotient over the coset g H_8n
// (quotient_poly.rs:52-58,115); the numerator has degree at most 5n + 6 (z times four wire
// factors) and t = num / Z_H at most 4n + 6, so any coset of more than 5n + 6 points
// interpolates the same t — bit-identical coefficients, commitments and proofs. This backend
// uses 6n points: g w3^m H_2n for m < 3 (w3 a primitive cube root of unity; gcd(3, 2n) = 1, so
// the three cosets form g H_6n), 25% fewer points than 8n. Every quotient-domain vector is
// laid out in three blocks of 2n (block m = coset m, natural order in u): evaluation point
// x(m, u) = s_m w_2n^u with s_m = g w3^m, the next row (w_n x) is u + 2 in the same block, and
// v_h(x) = x^n - 1 = g^n w3^(mn) (-1)^u - 1 takes 6 values (index 2m + (u & 1)).
constexpr int kQBlocks = 3;

struct QuotientArgs {
  const Fr *a, *b, *c, *d, *z, *pi, *l1, *sel, *sigma, *elements;  // pi null: no public inputs
  Fr* out;
  uint64_t nq;        // quotient-domain points (6n): kQBlocks blocks of 2n
  uint32_t log_blk;   // log2(2n)
  Fr g, alpha, alpha2, beta, gamma, k1, k2, k3;
  Fr range_sep, kappa, kappa2, kappa3;
  Fr logic_sep, lk, lk2, lk3, lk4;  // logic separation challenge and its kappa powers
  Fr fixed_sep, fk, fk2, fk3;        // fixed-base scalar mul: sep, kappa = sep^2, ^2, ^3
  Fr var_sep, vk, vk2;               // variable-base addition: sep, kappa = sep^2, ^2
  Fr edwards_d;                      // JubJub d = -10240/10241
  int has_range, has_logic, has_fixed, has_var;
  Fr vh_inv[2 * kQBlocks];  // 1 / v_h, index 2m + (u & 1)
  // k_quotient runs in the redundant form (ffr.hpp): a value with exponent e is stored as
  // x R 2^(-5e) (e = 0: the R domain; e = -1: the R' domain) and rx_mul adds exponents
  // plus one. Wire evaluations arrive at e = -1 (coset table scaled by 2^5), public
  // inputs at e = +1, z / selectors / sigmas / L1 / elements at e = 0; these constants are
  // pre-scaled so every term meets at e = 1 and num / v_h lands at e = 0 (the R domain).
  Fr rx_bg[kQBlocks], rx_beta, rx_gamma;  // beta s_m and beta at e = -2, gamma at e = -1
  Fr rx_one_w, rx_two_w, rx_three_w;    // 1, 2, 3 at e = -1 (range widget deltas)
  Fr rx_kappa, rx_kappa2, rx_kappa3;    // range kappa powers at e = -1
  Fr rx_alpha2;                         // alpha^2 at e = -1 (alpha and range_sep at e = 0)
  Fr rx_vh[2 * kQBlocks];               // 1 / v_h at e = -2
  Fr rx_inv32, rx_32;                   // 2^-5 and 2^5 (R domain): k_quotient_ext converts
};

constexpr int kMaxEval = 28;  // 16 proof evaluations + the linearisation terms at z
struct EvalBatch {
  const Fr* poly[kMaxEval];
  uint64_t len[kMaxEval];
  Fr x[kMaxEval];
};

constexpr int kMaxTerms = 24;  // the opening aggregate with r(X) expanded in place
struct LinComb {
  const Fr* p[kMaxTerms];
  uint64_t len[kMaxTerms];
  Fr s[kMaxTerms];
  uint32_t terms;
};

// delta_xor_and: 3(a + b + c) - 2 f + q_c (9c - 3(a + b)) with
// f = w (w (4w - 18(a + b) + 81) + 18(a^2 + b^2) - 81(a + b) + 83) = 6 (a AND b) for quads
PLK_HD Fr logic_xor_and(const Fr& a, const Fr& b, const Fr& w, const Fr& c,
                                            const Fr& qc) {
  auto k = [](uint32_t v) {
    Fr x = fe_zero<FrCfg>();
    x.v[0] = v;
    return fe_to_mont(x);
  };
  const Fr ab = fe_add(a, b);
  Fr f = fe_sub(fe_mul(k(4), w), fe_mul(k(18), ab));
  f = fe_add(f, k(81));
  f = fe_mul(w, f);
  f = fe_add(f, fe_mul(k(18), fe_add(fe_sqr(a), fe_sqr(b))));
  f = fe_sub(f, fe_mul(k(81), ab));
  f = fe_add(f, k(83));
  f = fe_mul(w, f);
  const Fr e = fe_sub(fe_mul(k(3), fe_add(ab, c)), fe_dbl(f));
  const Fr bb = fe_mul(qc, fe_sub(fe_mul(k(9), c), fe_mul(k(3), ab)));
  return fe_add(bb, e);
}

// Fixed-base scalar multiplication widget (dusk-plonk ecc/scalar_mul/fixed_base; zksnarks
// curve_scalar, un-vendored): accumulators (a, b) = point, d = scalar accumulator,
// c = xy_alpha, q_l / q_r / q_c = x_beta / y_beta / x_beta y_beta of the gate's multiple.
//   bit = d' - 2d;  bit (bit - 1)(bit + 1) + (bit q_c - c) k + x-check k^2 + y-check k^3
PLK_HD Fr widget_fixed_base(const Fr& ax, const Fr& ax_n, const Fr& ay, const Fr& ay_n,
                            const Fr& xy_alpha, const Fr& acc, const Fr& acc_n,
                            const Fr& x_beta, const Fr& y_beta, const Fr& xy_beta, const Fr& k,
                            const Fr& k2, const Fr& k3, const Fr& d) {
  const Fr one = fe_one<FrCfg>();
  const Fr bit = fe_sub(acc_n, fe_dbl(acc));
  const Fr bit_consistency = fe_mul(fe_mul(bit, fe_sub(bit, one)), fe_add(bit, one));
  const Fr y_alpha = fe_add(fe_mul(fe_sqr(bit), fe_sub(y_beta, one)), one);
  const Fr x_alpha = fe_mul(x_beta, bit);
  const Fr xy_consistency = fe_mul(fe_sub(fe_mul(bit, xy_beta), xy_alpha), k);
  const Fr prod = fe_mul(fe_mul(fe_mul(xy_alpha, ax), ay), d);
  const Fr x_lhs = fe_add(ax_n, fe_mul(ax_n, prod));
  const Fr x_rhs = fe_add(fe_mul(ax, y_alpha), fe_mul(ay, x_alpha));
  const Fr y_lhs = fe_sub(ay_n, fe_mul(ay_n, prod));
  const Fr y_rhs = fe_add(fe_mul(ay, y_alpha), fe_mul(ax, x_alpha));
  Fr id = fe_add(bit_consistency, xy_consistency);
  id = fe_add(id, fe_mul(fe_sub(x_lhs, x_rhs), k2));
  id = fe_add(id, fe_mul(fe_sub(y_lhs, y_rhs), k3));
  return id;
}

// Variable-base addition widget (dusk-plonk ecc/curve_addition; zksnarks curve_addtion):
// gate (x1, y1, x2, y2), next row (x3, y3, ., x1 y2):
//   (x1 y2 - x1y2') + (x1y2' + y1 x2 - x3 (1 + d x1y2' y1 x2)) k
//                   + (y1 y2 + x1 x2 - y3 (1 - d x1y2' y1 x2)) k^2
PLK_HD Fr widget_var_base(const Fr& x1, const Fr& x3, const Fr& y1, const Fr& y3, const Fr& x2,
                          const Fr& y2, const Fr& x1y2, const Fr& k, const Fr& k2, const Fr& d) {
  const Fr xy_consistency = fe_sub(fe_mul(x1, y2), x1y2);
  const Fr y1x2 = fe_mul(y1, x2);
  const Fr y1y2 = fe_mul(y1, y2);
  const Fr x1x2 = fe_mul(x1, x2);
  const Fr dprod = fe_mul(fe_mul(d, x1y2), y1x2);
  const Fr x3c = fe_sub(fe_add(x1y2, y1x2), fe_add(x3, fe_mul(x3, dprod)));
  const Fr y3c = fe_sub(fe_add(y1y2, x1x2), fe_sub(y3, fe_mul(y3, dprod)));
  return fe_add(fe_add(xy_consistency, fe_mul(x3c, k)), fe_mul(y3c, k2));
}

int pk_gather_wires(const Fr* witness, const uint32_t* idx, uint64_t m, uint64_t n, Fr* out,
                    hipStream_t s);
int pk_blind(Fr* poly, uint64_t n, const BlindArgs& b, hipStream_t s);
int pk_blind_batch(const BlindBatch& bb, uint64_t n, hipStream_t s);
// coefficients of PI(X) = idft(public-input vector) for at most kPiDirect public inputs:
// out[j] = sum_k c_k w^(-idx_k j), w^-e from the domain's R'-domain table tw_inv
int pk_pi_coef(const PiDirect& pd, const Fr* tw_inv, uint64_t n, Fr* out, hipStream_t s);
int pk_fill(Fr* out, const Fr& v, uint64_t n, hipStream_t s);
int pk_perm_numden(const Fr* wires, const Fr* sigmas, const Fr* elements, uint64_t n,
                   const Fr& beta, const Fr& gamma, const Fr& k1, const Fr& k2, const Fr& k3,
                   Fr* num, Fr* den, hipStream_t s);
int pk_mul3(const Fr* a, const Fr* b, const Fr& c, Fr* out, uint64_t n, hipStream_t s);
uint64_t pk_scan_tmp_elems(uint64_t n);
int pk_scan(const Fr* in, Fr* out, uint64_t n, bool mul, bool suffix, bool exclusive, Fr* tmp,
            hipStream_t s);
int pk_quotient(const QuotientArgs& q, hipStream_t s);
// t coefficients from the kQBlocks inverse block transforms B'_m (scaled by (2n)^-1 3^-1 s_m^-k):
// out[k + 2n l] = g^(-2nl) sum_m eta^(-ml) B'_m[k], eta = w3^(2n); comb = R'-domain constants
// {g^-2n, g^-2n eta^-1, g^-2n eta^-2, g^-4n, g^-4n eta^-2, g^-4n eta^-1}
int pk_coset3_combine(const Fr* in, uint64_t n2, const Fr* comb, Fr* out, hipStream_t s);
// out[j] = in[j] * c (packed Montgomery product), j < n
int pk_scale_copy(const Fr* in, const Fr& c, Fr* out, uint64_t n, hipStream_t s);
uint32_t pk_eval_max_blocks(uint64_t max_len);
int pk_eval(const EvalBatch& e, uint32_t count, uint64_t max_len, Fr* partial, Fr* d_out,
            hipStream_t s);
int pk_lincomb(const LinComb& lc, Fr* out, uint64_t len_out, hipStream_t s);
int pk_scale_powers(const Fr* c, uint64_t len, const Fr& x, uint64_t shift, Fr* y, hipStream_t s);
int pk_ruffini(const Fr* c, uint64_t len, const Fr& z, Fr* q, Fr* tmp, Fr* scan_tmp,
               hipStream_t s);

// ---- composer (host) ---------------------------------------------------------------
// One width-4 gate: q_m a b + q_l a + q_r b + q_o o + q_4 d + q_c + PI = 0 (lib.rs:546)
struct Gate {
  Fr q[11];  // q_m q_l q_r q_o q_4 q_c q_arith q_range q_logic q_fixed_group_add q_variable_group_add
  uint32_t w[4];  // a, b, o, d witness indices
  bool has_pi;
  Fr pi;
};

// The composer stores a gate as 24 bytes instead of Gate's 416: the four wires, a 2-bit
// code per selector (kSelZero / kSelOne / kSelMinusOne / kSelPooled) with bit kPiBit set
// when the gate carries a public input, and `ext`, the index in plk_composer::consts of
// the gate's pooled selectors (in selector order) followed by its PI value. Circuits are
// dominated by 0/±1 selectors, so synthesis writes ~17x fewer bytes per gate.
enum : uint32_t { kSelZero = 0, kSelOne = 1, kSelMinusOne = 2, kSelPooled = 3 };
constexpr uint32_t kPiBit = 1u << 22;
struct GateRec {
  uint32_t w[4];
  uint32_t code;
  uint32_t ext;
};
inline uint32_t sel_code(uint32_t code, int q) { return (code >> (2 * q)) & 3u; }

}  // namespace plk

struct plk_composer {
  std::vector<plk::Fr> witness;
  std::vector<plk::GateRec> gates;
  std::vector<plk::Fr> consts;  // pooled selector / PI values (see GateRec)
  // witness -> its wires in insertion order (permutation.rs:21-25,72-104), wire = 4*gate+col,
  // as flat singly linked lists (no per-witness allocation): head/tail per witness, next
  // per wire; kNoWire terminates.
  static constexpr uint32_t kNoWire = 0xffffffffu;
  std::vector<uint32_t> wire_head, wire_tail, wire_next;
  // running hash of the circuit's structure (every gate's wires, selector codes, pooled
  // selector values and public-input position — not witness or public-input values),
  // updated as gates are appended: plk_prove compares it with the key's in O(1)
  static constexpr uint64_t kHashInit = 0x6a09e667f3bcc908ull;
  uint64_t struct_hash = kHashInit;
};

struct plk_key {
  plk_ctx* ctx = nullptr;
  plk_srs* srs = nullptr;
  std::string label;
  uint64_t m = 0, n = 0, n_trim = 0;
  uint32_t k = 0;
  plk_domain* dom = nullptr;   // n
  plk_domain* domq = nullptr;  // 2n: the blocks of the 6n quotient domain (prover.hpp top)
  bool has_range = false, has_logic = false, has_fixed = false, has_var = false;
  // device-resident proving key
  plk::DevBuf q_coef;       // 11 x n selector coefficient polys
  plk::DevBuf selq;         // SEL_COUNTQ x 6n quotient-domain evaluations
  plk::DevBuf sigma_coef;   // 4 x n
  plk::DevBuf sigma_lag;    // 4 x n Lagrange values (= dft of sigma_coef, cached)
  plk::DevBuf sigmaq;       // 4 x 6n
  plk::DevBuf l1q;          // L1 over the quotient domain: coset_dft(idft(e_0)) (quotient_poly.rs:264-272)
  // forward coset tables, kQBlocks rows of n + 8 (R' domain): s_m^j for selectors, sigmas,
  // L1 and z; 2^5 s_m^j for the wires (evaluations at e = -1); 2^-5 s_m^j for PI (e = +1)
  plk::DevBuf coset_s, coset_w, coset_pi;
  plk::DevBuf icoset_q;     // kQBlocks rows of 2n: (2n)^-1 3^-1 s_m^-k (R'), inverse blocks
  plk::Fr s_m[plk::kQBlocks];    // g w3^m (R domain)
  plk::Fr comb[6];          // k_coset3_combine constants (R'): g^-2n w3'^-l m, l = 1, 2
  plk::DevBuf wire_idx;     // 4 x n witness indices per gate (u32)
  plk::Fr vh_inv[2 * plk::kQBlocks];
  plk_g1 comms[15];         // q_m q_l q_r q_o q_c q_4 q_arith q_range q_logic q_fixed q_var s1..s4
  // the circuit the key was compiled from: plk_prove refuses a circuit whose structure hash
  // differs or whose witness vector does not cover the largest wire index (prover.rs:114-119
  // reads the wires of the proving circuit; the key's gather indices must be valid for it)
  uint64_t struct_hash = 0;
  uint32_t max_wire = 0;
  // the prover behind plk_prove(key, ...) (context stream), created on first use
  std::mutex def_mu;
  std::unique_ptr<plk_prover> def_prover;
  ~plk_key();
};

// One concurrent prover over a key (include/plk.h plk_prover): stream, MSM workspace, NTT
// scratch and per-proof buffers of its own; the key and the SRS window table are shared
// read-only by every prover of the key.
struct plk_prover {
  plk_key* key = nullptr;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  plk::MsmWorkspace* ws = nullptr;  // owned (msm_workspace_new)
  // sharded commits (plk_prover_shard): this rank's SRS slice and the all-gather
  plk_srs* shard = nullptr;
  uint64_t shard_lo = 0;
  // plk_prover_shard_buckets (round 6): every commit on the key's own (whole) SRS, this rank
  // keeping bucket range `rank` of `world` (msm_run_batch part / parts) instead of a slice
  bool shard_buckets = false;
  int rank = 0, world = 1;
  plk_allgather_fn allgather = nullptr;
  void* allgather_user = nullptr;
  // per-proof scratch
  plk::PinnedBuf pin_witness, pin_small;  // host staging of the witness upload / small readbacks
  // the round-4 evaluations: coherent mapped host memory that k_eval_final writes directly
  plk::PinnedBuf eval_out;
  void* eval_dev = nullptr;  // eval_out's device address
  plk::DevBuf witness, wires_lag, wires_coef, z_lag, z_coef, num, den, tmp_a, scan_tmp, pi_lag,
      pi_coef, evq, quotq, t_coef, agg, agg2, w_coef, eval_partial, ntt_scratch;
  ~plk_prover();
};
