// prover.hip — host orchestration of the PLONK prover on the GPU: the composer (restating
// the reference's Plonk<C>, /root/reference/src/lib.rs), PlonkKey::compile_with_circuit
// (src/key.rs:63-327) and Prover::create_proof (src/prover.rs:67-474), with every O(n)
// step on the device (ntt.hip, msm.hip, prover_kernels.hip) and only the transcript and
// O(1) scalar algebra on the host.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <mutex>
#include <vector>

#include "ffr.hpp"
#include "internal.hpp"
#include "msm_common.hpp"
#include "prover.hpp"
#include "transcript.hpp"

using namespace plk;

namespace {

Fr fr_u64(uint64_t v) {
  Fr x = fe_zero<FrCfg>();
  x.v[0] = (uint32_t)v;
  x.v[1] = (uint32_t)(v >> 32);
  return fe_to_mont(x);
}
Fr fr_from(const plk_fr& a) {
  Fr r;
  for (int i = 0; i < 4; ++i) {
    r.v[2 * i] = (uint32_t)a.l[i];
    r.v[2 * i + 1] = (uint32_t)(a.l[i] >> 32);
  }
  return r;
}
plk_fr fr_to(const Fr& a) {
  plk_fr r;
  for (int i = 0; i < 4; ++i) r.l[i] = (uint64_t)a.v[2 * i] | ((uint64_t)a.v[2 * i + 1] << 32);
  return r;
}
bool fr_eq(const Fr& a, const Fr& b) { return fe_eq(a, b); }

// SplitMix64 -> uniform Fr (4 words, top masked to 255 bits, rejection), Montgomery out.
// The prover's randomness (blinding scalars) comes from an explicit seed so the CPU and
// GPU paths can consume identical randomness (SURVEY §7 hard part 5).
struct Rng {
  uint64_t s;
  uint64_t next() {
    s += 0x9E3779B97F4A7C15ull;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  Fr fr() {
    for (;;) {
      Fr c;
      for (int i = 0; i < 4; ++i) {
        const uint64_t w = next();
        c.v[2 * i] = (uint32_t)w;
        c.v[2 * i + 1] = (uint32_t)(w >> 32);
      }
      c.v[7] &= 0x7fffffffu;
      bool lt = false;
      for (int i = 7; i >= 0; --i)
        if (c.v[i] != FrCfg::P[i]) {
          lt = c.v[i] < FrCfg::P[i];
          break;
        }
      if (lt) return fe_to_mont(c);
    }
  }
  // uniform Fr drawn directly as its Montgomery image (x -> xR is a bijection of Fr), so no
  // multiply: used for the synthetic circuit's witnesses
  Fr fr_mont() {
    for (;;) {
      Fr c;
      for (int i = 0; i < 4; ++i) {
        const uint64_t w = next();
        c.v[2 * i] = (uint32_t)w;
        c.v[2 * i + 1] = (uint32_t)(w >> 32);
      }
      c.v[7] &= 0x7fffffffu;
      if (c.v[7] < FrCfg::P[7]) return c;  // top word strictly below: c < r
      if (c.v[7] == FrCfg::P[7]) {
        for (int i = 6; i >= 0; --i)
          if (c.v[i] != FrCfg::P[i]) {
            if (c.v[i] < FrCfg::P[i]) return c;
            break;
          }
      }
    }
  }
};

enum { QM = 0, QL, QR, QO, Q4, QC, QARITH, QRANGE, QLOGIC, QFIXED, QVAR };

Gate default_gate() {
  Gate g;
  for (auto& q : g.q) q = fe_zero<FrCfg>();
  for (auto& w : g.w) w = 0;  // Plonk::ZERO
  g.has_pi = false;
  g.pi = fe_zero<FrCfg>();
  return g;
}

uint32_t append_witness(plk_composer* c, const Fr& v) {
  c->witness.push_back(v);
  c->wire_head.push_back(plk_composer::kNoWire);
  c->wire_tail.push_back(plk_composer::kNoWire);
  return (uint32_t)(c->witness.size() - 1);
}

// Montgomery images of the selector codes kSelZero / kSelOne / kSelMinusOne
struct SelConsts {
  Fr v[3];
  SelConsts() {
    v[0] = fe_zero<FrCfg>();
    v[1] = fe_one<FrCfg>();
    v[2] = fe_neg(v[1]);
  }
};
const SelConsts& sel_consts() {
  static const SelConsts k;
  return k;
}

GateRec gate_pack(plk_composer* c, const Gate& g) {
  const SelConsts& k = sel_consts();
  GateRec r;
  std::memcpy(r.w, g.w, sizeof r.w);
  r.code = 0;
  r.ext = (uint32_t)c->consts.size();
  for (int q = 0; q < 11; ++q) {
    uint32_t code = kSelPooled;
    for (uint32_t j = 0; j < 3; ++j)
      if (fe_eq(g.q[q], k.v[j])) {
        code = j;
        break;
      }
    if (code == kSelPooled) c->consts.push_back(g.q[q]);
    r.code |= code << (2 * q);
  }
  if (g.has_pi) {
    r.code |= kPiBit;
    c->consts.push_back(g.pi);
  }
  return r;
}

Gate gate_unpack(const plk_composer* c, size_t i) {
  const SelConsts& k = sel_consts();
  const GateRec& r = c->gates[i];
  Gate g;
  std::memcpy(g.w, r.w, sizeof g.w);
  uint32_t e = r.ext;
  for (int q = 0; q < 11; ++q) {
    const uint32_t code = sel_code(r.code, q);
    g.q[q] = code == kSelPooled ? c->consts[e++] : k.v[code];
  }
  g.has_pi = (r.code & kPiBit) != 0;
  g.pi = g.has_pi ? c->consts[e] : fe_zero<FrCfg>();
  return g;
}

inline uint64_t hash_mix(uint64_t h, uint64_t v) {
  h ^= v + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
  return h * 0xff51afd7ed558ccdull;
}

int push_gate(plk_composer* c, const GateRec& g) {
  for (int k = 0; k < 4; ++k)
    if (g.w[k] >= c->witness.size()) return PLK_E_ARG;  // permutation.rs:98 assert
  const uint32_t n = (uint32_t)c->gates.size();
  c->gates.push_back(g);
  {  // structure hash: wires, selector codes (incl. the PI bit) and pooled selector values
    uint64_t h = hash_mix(c->struct_hash, (uint64_t)g.w[0] | ((uint64_t)g.w[1] << 32));
    h = hash_mix(h, (uint64_t)g.w[2] | ((uint64_t)g.w[3] << 32));
    h = hash_mix(h, g.code);
    uint32_t e = g.ext;
    for (int q = 0; q < 11; ++q)
      if (sel_code(g.code, q) == kSelPooled) {
        const Fr& v = c->consts[e++];
        for (int i = 0; i < 8; i += 2) h = hash_mix(h, (uint64_t)v.v[i] | ((uint64_t)v.v[i + 1] << 32));
      }
    c->struct_hash = h;
  }
  for (int k = 0; k < 4; ++k) {  // add_witnesses_to_map (permutation.rs:72-91)
    const uint32_t wire = 4 * n + k, wit = g.w[k];
    c->wire_next.push_back(plk_composer::kNoWire);
    if (c->wire_tail[wit] == plk_composer::kNoWire)
      c->wire_head[wit] = wire;
    else
      c->wire_next[c->wire_tail[wit]] = wire;
    c->wire_tail[wit] = wire;
  }
  return PLK_OK;
}

int append_custom_gate(plk_composer* c, const Gate& g) {
  for (int k = 0; k < 4; ++k)
    if (g.w[k] >= c->witness.size()) return PLK_E_ARG;
  return push_gate(c, gate_pack(c, g));
}

int append_gate(plk_composer* c, Gate g) {  // Constraint::arithmetic
  g.q[QARITH] = fe_one<FrCfg>();
  return append_custom_gate(c, g);
}

// append_evaluated_output (lib.rs:555-600): o = -(q_m a b + q_l a + q_r b + q_4 d + q_c + PI) / q_o
bool evaluated_output(plk_composer* c, const Gate& s, uint32_t& out) {
  const Fr a = c->witness[s.w[0]], b = c->witness[s.w[1]], d = c->witness[s.w[3]];
  Fr x = fe_mul(fe_mul(s.q[QM], a), b);
  x = fe_add(x, fe_mul(s.q[QL], a));
  x = fe_add(x, fe_mul(s.q[QR], b));
  x = fe_add(x, fe_mul(s.q[Q4], d));
  x = fe_add(x, s.q[QC]);
  if (s.has_pi) x = fe_add(x, s.pi);
  const Fr y = s.q[QO];
  if (fe_is_zero(y)) return false;
  Fr o;
  if (fr_eq(y, fe_one<FrCfg>()))
    o = fe_neg(x);
  else if (fr_eq(y, fe_neg(fe_one<FrCfg>())))
    o = x;
  else
    o = fe_mul(x, fe_neg(fe_inv(y)));
  out = append_witness(c, o);
  return true;
}

void assert_equal_constant(plk_composer* c, uint32_t a, const Fr& constant, const Fr* pi) {
  Gate g = default_gate();
  g.q[QL] = fe_one<FrCfg>();
  g.q[QC] = fe_neg(constant);
  g.w[0] = a;
  if (pi) {
    g.has_pi = true;
    g.pi = *pi;
  }
  (void)append_gate(c, g);
}

// lib.rs:606-640
void append_dummy_gates(plk_composer* c) {
  const uint32_t six = append_witness(c, fr_u64(6));
  const uint32_t one = append_witness(c, fr_u64(1));
  const uint32_t seven = append_witness(c, fr_u64(7));
  const uint32_t min_twenty = append_witness(c, fe_neg(fr_u64(20)));
  Gate g = default_gate();
  g.q[QM] = fr_u64(1);
  g.q[QL] = fr_u64(2);
  g.q[QR] = fr_u64(3);
  g.q[Q4] = fr_u64(1);
  g.q[QC] = fr_u64(4);
  g.q[QO] = fr_u64(4);
  g.w[0] = six;
  g.w[1] = seven;
  g.w[3] = one;
  g.w[2] = min_twenty;
  (void)append_gate(c, g);
  Gate h = default_gate();
  h.q[QM] = fr_u64(1);
  h.q[QL] = fr_u64(1);
  h.q[QR] = fr_u64(1);
  h.q[QC] = fr_u64(127);
  h.q[QO] = fr_u64(1);
  h.w[0] = min_twenty;
  h.w[1] = six;
  h.w[2] = seven;
  (void)append_gate(c, h);
}

Gate gate_from(const plk_constraint* s) {
  Gate g = default_gate();
  const plk_fr* qs[11] = {&s->q_m, &s->q_l, &s->q_r, &s->q_o, &s->q_4, &s->q_c, &s->q_arith,
                          &s->q_range, &s->q_logic, &s->q_fixed_group_add, &s->q_variable_group_add};
  for (int i = 0; i < 11; ++i) g.q[i] = fr_from(*qs[i]);
  g.w[0] = s->a;
  g.w[1] = s->b;
  g.w[2] = s->o;
  g.w[3] = s->d;
  g.has_pi = s->has_public != 0;
  g.pi = fr_from(s->public_input);
  return g;
}

uint32_t log2_ceil(uint64_t x) {
  uint32_t k = 0;
  while ((1ull << k) < x) ++k;
  return k;
}

#define TRY(...)                       \
  do {                                 \
    int _st = (__VA_ARGS__);           \
    if (_st != PLK_OK) return _st;     \
  } while (0)

// commit a batch of device polys against the key's trimmed SRS (key.rs:81-82): a poly whose
// non-zero part is longer than the trimmed SRS fails with PLK_E_DEGREE. `ws` / `s`: the
// calling prover's MSM workspace and stream.
int key_commit(plk_key* key, MsmWorkspace& ws, const std::vector<const Fr*>& ptrs,
               const std::vector<size_t>& lens, plk_g1* outs, int* statuses, hipStream_t s,
               size_t cap = SIZE_MAX) {
  const size_t max_points = std::min<size_t>(std::min<size_t>(key->srs->n, key->n_trim), cap);
  std::vector<size_t> use(lens.size());
  for (size_t i = 0; i < lens.size(); ++i) use[i] = std::min(lens[i], max_points);
  int overall = PLK_OK;
  for (size_t base = 0; base < ptrs.size(); base += kMaxSlots) {
    const size_t m = std::min<size_t>(kMaxSlots, ptrs.size() - base);
    const int r = msm_run_batch(key->srs, ws, ptrs.data() + base, use.data() + base,
                                lens.data() + base, m, outs + base,
                                statuses ? statuses + base : nullptr, s);
    if (r != PLK_OK && r != PLK_E_DEGREE) return r;
    if (r != PLK_OK) overall = r;
  }
  return overall;
}

// The same commit group split over the ranks of a sharded prover (plk_prover_shard, SURVEY
// §8e): this rank's MSMs over its SRS slice [lo, hi) of every polynomial, one all-gather
// of (13 point words + status) per commit, and the fold of the partial points in rank order.
// The last rank also checks the tail [max_points, len) for the degree error, wherever that
// tail starts relative to its slice (an SRS longer than the circuit's trimmed one puts the
// last slice past it). Every rank takes part in the exchange even when its own MSMs failed,
// so no rank waits forever on a collective the others left.
// Bucket-range form (plk_prover_shard_buckets, round 6): every rank holds the key's whole SRS
// and window table and runs each commit of the group over ALL of its points, keeping only the
// digits of bucket range `rank` of `world` (msm_run_batch part / parts: its sort, accumulation
// and run-sum / bit-sum reduction cover 1/world of the 2^(c-1) buckets); its outputs are that
// range's shares, and the same exchange and fold give the commitments. Every part checks the
// degree tail itself, so every rank sees the same status.
int shard_commit(plk_prover* P, const std::vector<const Fr*>& ptrs,
                 const std::vector<size_t>& lens, plk_g1* outs, int* statuses, size_t cap) {
  plk_key* key = P->key;
  const size_t cnt = ptrs.size();
  const size_t max_points = std::min<size_t>(std::min<size_t>(key->srs->n, key->n_trim), cap);
  const bool buckets = P->shard_buckets;
  plk_srs* srs = buckets ? key->srs : P->shard;
  const uint64_t lo = buckets ? 0 : P->shard_lo, hi = buckets ? key->srs->n : lo + P->shard->n;
  const bool last = buckets || P->rank == P->world - 1;
  const uint32_t part = buckets ? (uint32_t)P->rank : 0, parts = buckets ? (uint32_t)P->world : 1;
  std::vector<const Fr*> lp(cnt);
  std::vector<size_t> luse(cnt), lchk(cnt);
  int local = PLK_OK;
  if (last && hi < max_points) local = PLK_E_ARG;  // the slices do not cover the trimmed SRS
  for (size_t i = 0; i < cnt; ++i) {
    const size_t use = std::min(lens[i], max_points);
    luse[i] = use > lo ? (size_t)(std::min<uint64_t>(use, hi) - lo) : 0;
    lchk[i] = luse[i];
    lp[i] = ptrs[i] + lo;
    if (last && lens[i] > use) {
      if (use >= lo) {
        lchk[i] = lens[i] - lo;  // the tail follows this slice's own points
      } else {
        // nothing of this polynomial falls in the slice: an empty MSM whose base is the
        // start of the tail, so the degree check reads [use, lens) (no SRS point is read)
        lp[i] = ptrs[i] + use;
        lchk[i] = lens[i] - use;
      }
    }
  }
  std::vector<plk_g1> shares(cnt, plk_g1{});
  std::vector<int> pst(cnt, PLK_OK);
  for (size_t base = 0; local == PLK_OK && base < cnt; base += kMaxSlots) {
    const size_t m = std::min<size_t>(kMaxSlots, cnt - base);
    const int r = msm_run_batch(srs, *P->ws, lp.data() + base, luse.data() + base,
                                lchk.data() + base, m, shares.data() + base, pst.data() + base,
                                P->stream, part, parts);
    if (r != PLK_OK && r != PLK_E_DEGREE) local = r;
  }
  // payload per commit: x[6], y[6], infinity, status
  constexpr size_t kWords = 14;
  std::vector<uint64_t> send(cnt * kWords), recv((size_t)P->world * cnt * kWords);
  for (size_t i = 0; i < cnt; ++i) {
    uint64_t* w = &send[i * kWords];
    std::memcpy(w, &shares[i], sizeof(plk_g1));
    w[13] = (uint64_t)(local != PLK_OK ? local : pst[i]);
  }
  if (P->allgather(P->allgather_user, send.data(), send.size() * 8, recv.data()) != 0)
    return PLK_E_DEVICE;
  int overall = PLK_OK;
  std::vector<plk_g1> pts((size_t)P->world);
  for (size_t i = 0; i < cnt; ++i) {
    int st = PLK_OK;
    for (int r = 0; r < P->world; ++r) {
      const uint64_t* w = &recv[((size_t)r * cnt + i) * kWords];
      std::memcpy(&pts[r], w, sizeof(plk_g1));
      if (w[13] != PLK_OK && (st == PLK_OK || st == PLK_E_DEGREE)) st = (int)w[13];
    }
    if (st != PLK_OK && st != PLK_E_DEGREE) return st;  // a rank's device / argument error
    if (statuses) statuses[i] = st;
    if (st != PLK_OK) {
      outs[i] = plk_g1{};
      overall = PLK_E_DEGREE;
      continue;
    }
    const int r = plk_g1_sum(pts.data(), pts.size(), &outs[i]);
    if (r != PLK_OK) return r;
  }
  return overall;
}

// cap: commit at most `cap` points, the rest of each polynomial must be zero (else
// PLK_E_DEGREE) — the quotient chunks' bound below
int prover_commit(plk_prover* P, const std::vector<const Fr*>& ptrs,
                  const std::vector<size_t>& lens, plk_g1* outs, int* statuses,
                  size_t cap = SIZE_MAX) {
  if (P->shard || P->shard_buckets) return shard_commit(P, ptrs, lens, outs, statuses, cap);
  return key_commit(P->key, *P->ws, ptrs, lens, outs, statuses, P->stream, cap);
}

// a primitive cube root of unity in Fr: 7^((r-1)/3) = 0xac45a4010001a40200000000ffffffff
// (Montgomery form)
Fr cube_root_of_unity() {
  static const uint32_t w[8] = {0xffffffffu, 0x00000000u, 0x0001a402u, 0xac45a401u,
                                0u, 0u, 0u, 0u};
  Fr x;
  for (int i = 0; i < 8; ++i) x.v[i] = w[i];
  return fe_to_mont(x);
}

// JubJub twisted-Edwards d = -10240/10241 mod r
// (0x2a9318e74bfa2b48f5fd9207e6bd7fd4292d7f6d37579d2601065fd6d6343eb1), Montgomery form
Fr edwards_d() {
  static const uint32_t w[8] = {0xd6343eb1u, 0x01065fd6u, 0x37579d26u, 0x292d7f6du,
                                0xe6bd7fd4u, 0xf5fd9207u, 0x4bfa2b48u, 0x2a9318e7u};
  Fr x;
  for (int i = 0; i < 8; ++i) x.v[i] = w[i];
  return fe_to_mont(x);
}

Fr d2h_fr(const Fr* p, hipStream_t s) {
  thread_local PinnedBuf pin;
  if (pin.alloc(sizeof(Fr)) != PLK_OK) return fe_zero<FrCfg>();
  (void)hipMemcpyAsync(pin.ptr, p, sizeof(Fr), hipMemcpyDeviceToHost, s);
  (void)stream_wait(s);
  return *pin.as<Fr>();
}

}  // namespace

// sigma values k_col(next) * w^gate(next) from wire codes (4*gate + col)
namespace plk {
namespace {
__global__ void k_sigma_values(const uint32_t* __restrict__ codes, const Fr* __restrict__ el,
                               uint64_t n, Fr k1, Fr k2, Fr k3, Fr* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 4 * n) return;
  const uint32_t code = codes[i];
  const uint32_t g = code >> 2, col = code & 3;
  Fr v = el[g];
  if (col == 1) v = fe_mul(v, k1);
  if (col == 2) v = fe_mul(v, k2);
  if (col == 3) v = fe_mul(v, k3);
  out[i] = v;
}
}  // namespace
}  // namespace plk

extern "C" {

// ----------------------------------------------------------------------- composer
// Composer storage pool: a proof server synthesizes a fresh composer per proof (as
// create_proof does, prover.rs:76-78); reusing the vectors of destroyed composers (clear()
// keeps capacity) avoids re-faulting ~120 bytes of fresh pages per gate every proof.
namespace {
std::mutex g_pool_mu;
std::vector<std::unique_ptr<plk_composer>> g_pool;
constexpr size_t kPoolMax = 2;

std::unique_ptr<plk_composer> composer_from_pool() {
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    if (!g_pool.empty()) {
      std::unique_ptr<plk_composer> c = std::move(g_pool.back());
      g_pool.pop_back();
      return c;
    }
  }
  return std::unique_ptr<plk_composer>(new plk_composer());
}
}  // namespace

int plk_composer_create(plk_composer** out) {
  try {
    if (!out) return PLK_E_ARG;
    std::unique_ptr<plk_composer> c = composer_from_pool();
    // Plonk::initialize (lib.rs:121-134)
    const uint32_t zero = append_witness(c.get(), fe_zero<FrCfg>());
    const uint32_t one = append_witness(c.get(), fe_one<FrCfg>());
    assert_equal_constant(c.get(), zero, fe_zero<FrCfg>(), nullptr);
    assert_equal_constant(c.get(), one, fe_one<FrCfg>(), nullptr);
    append_dummy_gates(c.get());
    append_dummy_gates(c.get());
    *out = c.release();
    return PLK_OK;
  } catch (...) {
    return PLK_E_OOM;
  }
}

int plk_composer_destroy(plk_composer* c) {
  if (!c) return PLK_OK;
  std::unique_ptr<plk_composer> h(c);
  h->witness.clear();
  h->gates.clear();
  h->consts.clear();
  h->wire_head.clear();
  h->wire_tail.clear();
  h->wire_next.clear();
  h->struct_hash = plk_composer::kHashInit;
  std::lock_guard<std::mutex> lk(g_pool_mu);
  if (g_pool.size() < kPoolMax) g_pool.push_back(std::move(h));
  return PLK_OK;
}

int plk_composer_size(const plk_composer* c, size_t* gates, size_t* witnesses) {
  if (!c) return PLK_E_ARG;
  if (gates) *gates = c->gates.size();
  if (witnesses) *witnesses = c->witness.size();
  return PLK_OK;
}

int plk_composer_append_witness(plk_composer* c, const plk_fr* v, uint32_t* wire) {
  if (!c || !v || !wire) return PLK_E_ARG;
  *wire = append_witness(c, fr_from(*v));
  return PLK_OK;
}

int plk_composer_witness_value(const plk_composer* c, uint32_t wire, plk_fr* v) {
  if (!c || !v || wire >= c->witness.size()) return PLK_E_ARG;
  *v = fr_to(c->witness[wire]);
  return PLK_OK;
}

// lib.rs:708-719: witness + assert_equal_constant(w, 0, Some(-public))
int plk_composer_append_public(plk_composer* c, const plk_fr* v, uint32_t* wire) {
  if (!c || !v || !wire) return PLK_E_ARG;
  const Fr val = fr_from(*v);
  *wire = append_witness(c, val);
  const Fr neg = fe_neg(val);
  assert_equal_constant(c, *wire, fe_zero<FrCfg>(), &neg);
  return PLK_OK;
}

int plk_composer_append_gate(plk_composer* c, const plk_constraint* s) {
  if (!c || !s) return PLK_E_ARG;
  return append_gate(c, gate_from(s));
}

int plk_composer_append_custom_gate(plk_composer* c, const plk_constraint* s) {
  if (!c || !s) return PLK_E_ARG;
  return append_custom_gate(c, gate_from(s));
}

// lib.rs:1169-1197: q_o = -1, o := evaluated output, append
int plk_composer_gate_eval(plk_composer* c, const plk_constraint* s, uint32_t* out) {
  if (!c || !s || !out) return PLK_E_ARG;
  Gate g = gate_from(s);
  g.q[QARITH] = fe_one<FrCfg>();
  g.q[QO] = fe_neg(fe_one<FrCfg>());
  for (int k = 0; k < 4; ++k)
    if (g.w[k] >= c->witness.size() && k != 2) return PLK_E_ARG;
  uint32_t o;
  if (!evaluated_output(c, g, o)) return PLK_E_ARG;
  g.w[2] = o;
  *out = o;
  return append_gate(c, g);
}

int plk_composer_assert_equal(plk_composer* c, uint32_t a, uint32_t b) {
  if (!c || a >= c->witness.size() || b >= c->witness.size()) return PLK_E_ARG;
  Gate g = default_gate();  // lib.rs:721-730
  g.q[QL] = fe_one<FrCfg>();
  g.q[QR] = fe_neg(fe_one<FrCfg>());
  g.w[0] = a;
  g.w[1] = b;
  return append_gate(c, g);
}

int plk_composer_assert_equal_constant(plk_composer* c, uint32_t a, const plk_fr* constant,
                                       const plk_fr* public_input) {
  if (!c || !constant || a >= c->witness.size()) return PLK_E_ARG;
  const Fr pi = public_input ? fr_from(*public_input) : fe_zero<FrCfg>();
  assert_equal_constant(c, a, fr_from(*constant), public_input ? &pi : nullptr);
  return PLK_OK;
}

// component_range (lib.rs:1066-1163): base-4 accumulators over the witness's canonical bits
// (LSB first), 4 quads per width-4 gate with q_range = 1 (d, o, b, a order within a gate,
// the next gate's d closing the chain), a final zero-selector gate carrying the last
// accumulator, and the last accumulator asserted equal to the witness.
int plk_composer_component_range(plk_composer* c, uint32_t witness, size_t num_bits) {
  if (!c || witness >= c->witness.size() || num_bits > 256) return PLK_E_ARG;
  try {
    const Fr canon = fe_from_mont(c->witness[witness]);
    auto bit = [&](size_t i) -> uint32_t { return (canon.v[i / 32] >> (i % 32)) & 1u; };
    size_t num_gates = num_bits >> 3;
    if (num_bits % 8 != 0) ++num_gates;
    const size_t num_quads = num_gates * 4;
    const size_t pad = 1 + (((num_quads << 1) - num_bits) >> 1);
    Gate base = default_gate();
    base.q[QRANGE] = fe_one<FrCfg>();  // Constraint::range
    std::vector<Gate> cons(num_gates + 1, base);
    std::vector<uint32_t> accs;
    const Fr four = fr_u64(4);
    Fr acc = fe_zero<FrCfg>();
    for (size_t i = pad; i <= num_quads; ++i) {
      const size_t bi = (num_quads - i) << 1;
      const uint32_t quad = (bi < 256 ? bit(bi) : 0u) + 2 * (bi + 1 < 256 ? bit(bi + 1) : 0u);
      acc = fe_add(fe_mul(four, acc), fr_u64(quad));
      const uint32_t w = append_witness(c, acc);
      accs.push_back(w);
      Gate& g = cons[i / 4];
      switch (i % 4) {
        case 0: g.w[3] = w; break;
        case 1: g.w[2] = w; break;
        case 2: g.w[1] = w; break;
        default: g.w[0] = w; break;
      }
    }
    cons.back() = default_gate();
    if (!accs.empty()) cons.back().w[3] = accs.back();
    for (const Gate& g : cons)
      if (append_custom_gate(c, g) != PLK_OK) return PLK_E_ARG;
    if (!accs.empty()) return plk_composer_assert_equal(c, accs.back(), witness);
    return PLK_OK;
  } catch (...) {
    return PLK_E_OOM;
  }
}

int plk_composer_component_boolean(plk_composer* c, uint32_t a) {
  if (!c || a >= c->witness.size()) return PLK_E_ARG;
  Gate g = default_gate();  // lib.rs:859-872
  g.q[QM] = fe_one<FrCfg>();
  g.q[QO] = fe_neg(fe_one<FrCfg>());
  g.w[0] = a;
  g.w[1] = a;
  g.w[2] = a;
  g.w[3] = 0;
  return append_gate(c, g);
}

// The bench circuit: `gates` arithmetic gates of the chain
// x_{i+1} = x_i * y_i + x_i via gate_mul-style gates (q_m = 1, q_l = 1, q_o = -1) whose
// outputs feed the next gate's a-wire (non-trivial copy constraints); y_i from SplitMix64.
int plk_composer_synthetic_chain(plk_composer* c, size_t gates, uint64_t seed) {
  if (!c) return PLK_E_ARG;
  try {
    Rng rng{seed};
    uint32_t x = append_witness(c, rng.fr_mont());
    c->witness.reserve(c->witness.size() + 2 * gates);
    c->wire_head.reserve(c->wire_head.size() + 2 * gates);
    c->wire_tail.reserve(c->wire_tail.size() + 2 * gates);
    c->wire_next.reserve(c->wire_next.size() + 4 * gates);
    c->gates.reserve(c->gates.size() + gates);
    GateRec g;
    g.code = (kSelOne << (2 * QM)) | (kSelOne << (2 * QL)) | (kSelMinusOne << (2 * QO)) |
             (kSelOne << (2 * QARITH));
    g.ext = (uint32_t)c->consts.size();
    g.w[3] = 0;  // Plonk::ZERO
    for (size_t i = 0; i < gates; ++i) {
      const uint32_t y = append_witness(c, rng.fr_mont());
      const Fr& xv = c->witness[x];
      const Fr o = fe_add(fe_mul(xv, c->witness[y]), xv);
      g.w[0] = x;
      g.w[1] = y;
      g.w[2] = append_witness(c, o);
      if (push_gate(c, g) != PLK_OK) return PLK_E_ARG;
      x = g.w[2];
    }
    return PLK_OK;
  } catch (...) {
    return PLK_E_OOM;
  }
}

// Overwrite witness values (a new instance of the same circuit, as create_proof
// re-synthesizes the circuit with new witnesses, prover.rs:76-78).
int plk_composer_set_witness(plk_composer* c, uint32_t wire, const plk_fr* v) {
  if (!c || !v || wire >= c->witness.size()) return PLK_E_ARG;
  c->witness[wire] = fr_from(*v);
  return PLK_OK;
}

// public inputs, sorted by gate index (Plonk::instance, lib.rs:182-196)
int plk_composer_public_inputs(const plk_composer* c, plk_fr* values, uint64_t* indexes,
                               size_t cap, size_t* count) {
  if (!c || !count) return PLK_E_ARG;
  size_t k = 0;
  for (size_t i = 0; i < c->gates.size(); ++i) {
    if (!(c->gates[i].code & kPiBit)) continue;
    if (k < cap) {
      if (values) values[k] = fr_to(gate_unpack(c, i).pi);
      if (indexes) indexes[k] = i;
    }
    ++k;
  }
  *count = k;
  return PLK_OK;
}

int plk_composer_export(const plk_composer* c, plk_constraint* gates, size_t cap,
                        plk_fr* witness, size_t wcap, size_t* m, size_t* nw) {
  if (!c) return PLK_E_ARG;
  if (m) *m = c->gates.size();
  if (nw) *nw = c->witness.size();
  if (gates) {
    const size_t cnt = std::min(cap, c->gates.size());
    for (size_t i = 0; i < cnt; ++i) {
      const Gate g = gate_unpack(c, i);
      plk_constraint& o = gates[i];
      plk_fr* qs[11] = {&o.q_m,     &o.q_l,   &o.q_r,     &o.q_o,
                        &o.q_4,     &o.q_c,   &o.q_arith, &o.q_range,
                        &o.q_logic, &o.q_fixed_group_add, &o.q_variable_group_add};
      for (int q = 0; q < 11; ++q) *qs[q] = fr_to(g.q[q]);
      o.a = g.w[0];
      o.b = g.w[1];
      o.o = g.w[2];
      o.d = g.w[3];
      o.has_public = g.has_pi ? 1u : 0u;
      o._pad = 0;
      o.public_input = fr_to(g.pi);
    }
  }
  if (witness) {
    const size_t cnt = std::min(wcap, c->witness.size());
    for (size_t j = 0; j < cnt; ++j) witness[j] = fr_to(c->witness[j]);
  }
  return PLK_OK;
}

// ---------------------------------------------------------------------------- key
int plk_key_compile(plk_srs* srs, const plk_composer* cs, const char* label, plk_key** out) {
  try {
    if (!srs || !cs || !out) return PLK_E_ARG;
    *out = nullptr;
    plk_ctx* ctx = srs->ctx;
    DeviceGuard guard(ctx->device);
    hipStream_t s = ctx->stream;
    std::unique_ptr<plk_key> key(new plk_key());
    key->ctx = ctx;
    key->srs = srs;
    key->label = label ? label : "plonk";
    const uint64_t m = cs->gates.size();
    const uint32_t k = log2_ceil(m);
    const uint64_t n = 1ull << k;
    key->m = m;
    key->n = n;
    key->k = k;
    // keypair.trim(additional_n) with additional_n = next_pow2(m + 6) (key.rs:81-82); the
    // trimmed SRS keeps PlonkParams' slack of 8 points
    key->n_trim = (1ull << log2_ceil(m + 6)) + 8;
    if (k + 1 > 27) return PLK_E_ARG;
    for (uint64_t i = 0; i < m; ++i) {
      const Gate g = gate_unpack(cs, i);
      if (!fe_is_zero(g.q[QRANGE])) key->has_range = true;
      if (!fe_is_zero(g.q[QLOGIC])) key->has_logic = true;
      if (!fe_is_zero(g.q[QFIXED])) key->has_fixed = true;
      if (!fe_is_zero(g.q[QVAR])) key->has_var = true;
    }
    TRY(plk_domain_get(ctx, k, &key->dom));
    TRY(plk_domain_get(ctx, k + 1, &key->domq));
    const uint64_t n2 = 2 * n, nq = kQBlocks * n2;

    // 1. selectors padded to n (key.rs:89-119) -> idft (key.rs:121-131)
    std::vector<Fr> host(11 * n, fe_zero<FrCfg>());
    for (uint64_t i = 0; i < m; ++i) {
      const Gate g = gate_unpack(cs, i);
      for (int q = 0; q < 11; ++q) host[q * n + i] = g.q[q];
    }
    TRY(key->q_coef.alloc(11 * n * sizeof(Fr)));
    PLK_HIP_TRY(hipMemcpyAsync(key->q_coef.ptr, host.data(), 11 * n * sizeof(Fr),
                               hipMemcpyHostToDevice, s));
    Fr* qc = key->q_coef.as<Fr>();
    for (int q = 0; q < 11; ++q) TRY(ntt_run(key->dom, qc + q * n, qc + q * n, n, -1, 0, nullptr, s, 1));

    // 2. sigma permutations (permutation.rs:108-141) and Lagrange encodings (:143-168)
    std::vector<uint32_t> codes(4 * n);
    for (uint64_t i = 0; i < n; ++i)
      for (uint32_t col = 0; col < 4; ++col) codes[col * n + i] = (uint32_t)(4 * i + col);
    // each witness's wires form a cycle in insertion order: wire -> next, last -> first
    for (size_t wit = 0; wit < cs->wire_head.size(); ++wit)
      for (uint32_t cur = cs->wire_head[wit]; cur != plk_composer::kNoWire; cur = cs->wire_next[cur]) {
        const uint32_t nx = cs->wire_next[cur];
        const uint32_t nxt = nx == plk_composer::kNoWire ? cs->wire_head[wit] : nx;
        codes[(cur & 3) * n + (cur >> 2)] = nxt;
      }
    DevBuf dcodes;
    TRY(dcodes.alloc(4 * n * 4));
    PLK_HIP_TRY(hipMemcpyAsync(dcodes.ptr, codes.data(), 4 * n * 4, hipMemcpyHostToDevice, s));
    TRY(key->sigma_lag.alloc(4 * n * sizeof(Fr)));
    hipLaunchKernelGGL(k_sigma_values, dim3((unsigned)((4 * n + 255) / 256)), dim3(256), 0, s,
                       dcodes.as<uint32_t>(), key->dom->tw_fwd.as<Fr>(), n, fr_u64(7), fr_u64(13),
                       fr_u64(17), key->sigma_lag.as<Fr>());
    PLK_HIP_TRY(hipGetLastError());
    TRY(key->sigma_coef.alloc(4 * n * sizeof(Fr)));
    Fr* sc = key->sigma_coef.as<Fr>();
    for (int c = 0; c < 4; ++c)
      TRY(ntt_run(key->dom, key->sigma_lag.as<Fr>() + c * n, sc + c * n, n, -1, 0, nullptr, s, 1));

    // 3. commitments (key.rs:138-159): selectors swallow errors, sigmas propagate
    const int order[11] = {QM, QL, QR, QO, QC, Q4, QARITH, QRANGE, QLOGIC, QFIXED, QVAR};
    std::vector<const Fr*> ptrs;
    std::vector<size_t> lens;
    for (int q : order) {
      ptrs.push_back(qc + q * n);
      lens.push_back(n);
    }
    for (int c = 0; c < 4; ++c) {
      ptrs.push_back(sc + c * n);
      lens.push_back(n);
    }
    int sts[15];
    const int r = key_commit(key.get(), *srs->ws, ptrs, lens, key->comms, sts, s);
    if (r != PLK_OK && r != PLK_E_DEGREE) return r;
    for (int i = 0; i < 11; ++i)
      if (sts[i] != PLK_OK) key->comms[i] = plk_g1{{0}, {0}, 1};  // unwrap_or_default
    for (int i = 11; i < 15; ++i)
      if (sts[i] != PLK_OK) return sts[i];

    // 4. quotient-domain evaluations (key.rs:220-245 over g H_8n there; g H_6n here, see
    // prover.hpp) and v_h over it (key.rs:291)
    {
      const Fr gq = key->domq->g, one = fe_one<FrCfg>();
      const Fr w3 = cube_root_of_unity();
      const uint64_t rowc = n + 8;  // coset table row: the transforms read <= n + 3 inputs
      TRY(key->coset_s.alloc(kQBlocks * rowc * sizeof(Fr)));
      TRY(key->coset_w.alloc(kQBlocks * rowc * sizeof(Fr)));
      TRY(key->coset_pi.alloc(kQBlocks * rowc * sizeof(Fr)));
      TRY(key->icoset_q.alloc(kQBlocks * n2 * sizeof(Fr)));
      const Fr c32 = fr_u64(32), inv3 = fe_inv(fr_u64(3));
      Fr sm = gq;
      for (int mb = 0; mb < kQBlocks; ++mb) {
        key->s_m[mb] = sm;
        TRY(ntt_power_table(key->coset_s.as<Fr>() + mb * rowc, sm, one, rowc, true, s));
        TRY(ntt_power_table(key->coset_w.as<Fr>() + mb * rowc, sm, c32, rowc, true, s));
        TRY(ntt_power_table(key->coset_pi.as<Fr>() + mb * rowc, sm, fe_inv(c32), rowc, true, s));
        TRY(ntt_power_table(key->icoset_q.as<Fr>() + mb * n2, fe_inv(sm),
                            fe_mul(key->domq->n_inv, inv3), n2, true, s));
        sm = fe_mul(sm, w3);
      }
      // k_coset3_combine: c[k + 2n l] = g^(-2nl) sum_m eta^(-ml) B'_m[k], eta = w3^(2n)
      const Fr eta_inv = fe_inv(fe_pow_u64(w3, n2));
      const Fr eta_inv2 = fe_sqr(eta_inv);
      const Fr g1 = fe_inv(fe_pow_u64(gq, n2)), g2 = fe_sqr(g1);
      const Fr cm[6] = {g1, fe_mul(g1, eta_inv), fe_mul(g1, eta_inv2),
                        g2, fe_mul(g2, eta_inv2), fe_mul(g2, eta_inv)};
      for (int j = 0; j < 6; ++j) key->comb[j] = fe_to_rx_domain(cm[j]);
      // v_h(s_m w_2n^u) = g^n w3^(mn) (-1)^u - 1: index 2m + (u & 1)
      for (int mb = 0; mb < kQBlocks; ++mb) {
        const Fr x = fe_pow_u64(key->s_m[mb], n);
        key->vh_inv[2 * mb] = fe_inv(fe_sub(x, one));
        key->vh_inv[2 * mb + 1] = fe_inv(fe_sub(fe_neg(x), one));
      }
    }
    // forward coset transforms of n-coefficient polys onto the three blocks in one launch
    auto coset_fwd = [&](const Fr* in, Fr* out, uint64_t len, const DevBuf& table) {
      NttBatch b;
      b.in_stride = 0;  // the same coefficients for every block
      b.out_stride = n2;
      b.pre = table.as<Fr>();
      b.pre_stride = n + 8;
      return ntt_run_batch(key->domq, in, out, len, 1, 1, nullptr, s, kQBlocks, b);
    };
    TRY(key->selq.alloc(SEL_COUNTQ * nq * sizeof(Fr)));
    const int sel_src[SEL_COUNTQ] = {QM, QL, QR, QO, Q4, QC, QARITH, QRANGE, QLOGIC, QFIXED, QVAR};
    const bool sel_used[SEL_COUNTQ] = {true, true, true, true, true, true, true, key->has_range,
                                       key->has_logic, key->has_fixed, key->has_var};
    for (int j = 0; j < SEL_COUNTQ; ++j)  // unused widget selectors are never read
      if (sel_used[j])
        TRY(coset_fwd(qc + sel_src[j] * n, key->selq.as<Fr>() + j * nq, n, key->coset_s));
    TRY(key->sigmaq.alloc(4 * nq * sizeof(Fr)));
    for (int c = 0; c < 4; ++c)
      TRY(coset_fwd(sc + c * n, key->sigmaq.as<Fr>() + c * nq, n, key->coset_s));
    // L1 over the quotient domain, shared by every proof: idft(e_0) = n^-1 in every coefficient
    TRY(key->l1q.alloc(nq * sizeof(Fr)));
    {
      DevBuf tmp;
      TRY(tmp.alloc(n * sizeof(Fr)));
      TRY(pk_fill(tmp.as<Fr>(), key->dom->n_inv, n, s));
      TRY(coset_fwd(tmp.as<Fr>(), key->l1q.as<Fr>(), n, key->coset_s));
      PLK_HIP_TRY(stream_wait(s));
    }
    // 5. wire indices for the per-proof gather (prover.rs:114-119)
    std::vector<uint32_t> idx(4 * n, 0);
    for (uint64_t i = 0; i < m; ++i)
      for (int c = 0; c < 4; ++c) {
        idx[c * n + i] = cs->gates[i].w[c];
        key->max_wire = std::max(key->max_wire, cs->gates[i].w[c]);
      }
    key->struct_hash = cs->struct_hash;
    TRY(key->wire_idx.alloc(4 * n * 4));
    PLK_HIP_TRY(hipMemcpyAsync(key->wire_idx.ptr, idx.data(), 4 * n * 4, hipMemcpyHostToDevice, s));
    PLK_HIP_TRY(stream_wait(s));
    *out = key.release();
    return PLK_OK;
  } catch (const std::bad_alloc&) {
    return PLK_E_OOM;
  } catch (...) {
    return PLK_E_DEVICE;
  }
}

int plk_key_destroy(plk_key* key) {
  if (!key) return PLK_E_ARG;
  DeviceGuard g(key->ctx->device);
  (void)stream_wait(key->ctx->stream);
  delete key;
  return PLK_OK;
}

int plk_key_info(const plk_key* key, uint64_t* n, uint64_t* m, plk_g1* commitments) {
  if (!key) return PLK_E_ARG;
  if (n) *n = key->n;
  if (m) *m = key->m;
  if (commitments) std::memcpy(commitments, key->comms, sizeof key->comms);
  return PLK_OK;
}

// ----------------------------------------------------------------------- prover
int plk_prover_create(plk_key* key, plk_prover** out) {
  try {
    if (!key || !out) return PLK_E_ARG;
    *out = nullptr;
    DeviceGuard guard(key->ctx->device);
    std::unique_ptr<plk_prover> p(new plk_prover());
    p->key = key;
    p->ws = msm_workspace_new();
    // a lane shares the chip with other lanes' proofs: the reduction trees' form by circuit
    // size (msm_common.hpp lane_tail_policy, with the measured rows)
    if (!p->ws->tail_forced) p->ws->tail_quad = lane_tail_policy(key->n);
    p->ws->shared_chip = true;
    PLK_HIP_TRY(hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking));
    p->own_stream = true;
    *out = p.release();
    return PLK_OK;
  } catch (const std::bad_alloc&) {
    return PLK_E_OOM;
  }
}

int plk_prover_destroy(plk_prover* p) {
  if (!p) return PLK_E_ARG;
  DeviceGuard g(p->key->ctx->device);
  (void)stream_wait(p->stream);
  delete p;
  return PLK_OK;
}

int plk_prover_stream(plk_prover* p, void** stream_out) {
  if (!p || !stream_out) return PLK_E_ARG;
  *stream_out = p->stream;
  return PLK_OK;
}

int plk_prover_msm_stats(plk_prover* p, int reset, double* accumulate_ms, uint64_t* launches,
                         uint64_t* point_adds, uint64_t* points) {
  if (!p) return PLK_E_ARG;
  MsmStats& st = msm_workspace_stats(*p->ws);
  if (accumulate_ms) *accumulate_ms = st.cum_accumulate_ms;
  if (launches) *launches = st.cum_launches;
  if (point_adds) *point_adds = st.cum_point_adds;
  if (points) *points = st.cum_points;
  if (reset) st.reset_cum();
  return PLK_OK;
}

int plk_prover_shard(plk_prover* p, plk_srs* slice, uint64_t slice_start, int rank, int world,
                     plk_allgather_fn allgather, void* user) {
  if (!p || world < 1 || rank < 0 || rank >= world) return PLK_E_ARG;
  // world 1 with a slice and an all-gather still takes the exchange path (one slice covering
  // the SRS, one rank's partials exchanged): the whole sharded code path on one GPU. World 1
  // without them is the unsharded prover.
  const bool sharded = world > 1 || (slice && allgather);
  if (sharded && (!slice || !allgather || slice->ctx->device != p->key->ctx->device))
    return PLK_E_ARG;
  p->shard = sharded ? slice : nullptr;
  p->shard_lo = sharded ? slice_start : 0;
  p->shard_buckets = false;
  p->rank = rank;
  p->world = world;
  p->allgather = sharded ? allgather : nullptr;
  p->allgather_user = user;
  return PLK_OK;
}

int plk_prover_shard_buckets(plk_prover* p, int rank, int world, plk_allgather_fn allgather,
                             void* user) {
  if (!p || !allgather || world < 1 || rank < 0 || rank >= world) return PLK_E_ARG;
  // msm_run_batch's part conditions (a power of two; a wide bucket set, c >= 17, with >= 2^14
  // buckets per part); otherwise the caller keeps SRS slices (parallel.shard_prover_lane
  // mode "auto")
  if (!msm_parts_ok(p->key->srs, (uint32_t)world)) return PLK_E_ARG;
  p->shard = nullptr;
  p->shard_lo = 0;
  p->shard_buckets = true;
  p->rank = rank;
  p->world = world;
  p->allgather = allgather;
  p->allgather_user = user;
  return PLK_OK;
}

int plk_prove(plk_key* key, const plk_composer* cs, uint64_t seed, plk_proof* proof,
              plk_fr* public_inputs, size_t pi_cap, size_t* pi_count) {
  if (!key) return PLK_E_ARG;
  // the default prover's scratch, workspace and stream serve one proof at a time: concurrent
  // plk_prove calls on one key run one after the other (plk_prover_create gives parallel lanes)
  std::lock_guard<std::mutex> lk(key->def_mu);
  if (!key->def_prover) {
    try {
      std::unique_ptr<plk_prover> d(new plk_prover());
      d->key = key;
      d->ws = msm_workspace_new();
      d->stream = key->ctx->stream;  // the context's stream, not owned
      key->def_prover = std::move(d);
    } catch (const std::bad_alloc&) {
      return PLK_E_OOM;
    }
  }
  return plk_prover_prove(key->def_prover.get(), cs, seed, proof, public_inputs, pi_cap, pi_count);
}

int plk_prover_prove(plk_prover* P, const plk_composer* cs, uint64_t seed, plk_proof* proof,
                     plk_fr* public_inputs, size_t pi_cap, size_t* pi_count) {
  try {
    if (!P || !cs || !proof) return PLK_E_ARG;
    plk_key* key = P->key;
    // the proving circuit must have the key's structure (prover.rs:114-119 gathers the
    // wires of this circuit; the key's gather indices stand for them)
    if (cs->gates.size() != key->m || cs->struct_hash != key->struct_hash) return PLK_E_ARG;
    if (cs->witness.size() <= key->max_wire) return PLK_E_ARG;
    DeviceGuard guard(key->ctx->device);
    hipStream_t s = P->stream;
    const uint64_t n = key->n, m = key->m, S = n + 8;  // S: padded poly stride
    const uint64_t n2 = 2 * n, nq = kQBlocks * n2;       // quotient domain (prover.hpp)
    Rng rng{seed};
    const Fr one = fe_one<FrCfg>();
    const Fr K1 = fr_u64(7), K2 = fr_u64(13), K3 = fr_u64(17);

    // scratch (allocated once per prover)
    TRY(P->witness.alloc(std::max<size_t>(cs->witness.size(), 1) * sizeof(Fr)));
    TRY(P->wires_lag.alloc(4 * n * sizeof(Fr)));
    TRY(P->wires_coef.alloc(4 * S * sizeof(Fr)));
    TRY(P->z_lag.alloc(n * sizeof(Fr)));
    TRY(P->z_coef.alloc(S * sizeof(Fr)));
    TRY(P->num.alloc(n * sizeof(Fr)));
    TRY(P->den.alloc(n * sizeof(Fr)));
    TRY(P->scan_tmp.alloc((pk_scan_tmp_elems(5 * n) + 1) * sizeof(Fr)));
    TRY(P->pi_lag.alloc(n * sizeof(Fr)));
    TRY(P->pi_coef.alloc(n * sizeof(Fr)));
    TRY(P->evq.alloc(6 * nq * sizeof(Fr)));
    TRY(P->quotq.alloc(nq * sizeof(Fr)));
    TRY(P->t_coef.alloc(nq * sizeof(Fr)));
    TRY(P->agg.alloc(5 * n * sizeof(Fr)));
    TRY(P->agg2.alloc(S * sizeof(Fr)));
    TRY(P->w_coef.alloc((5 * n + S) * sizeof(Fr)));
    TRY(P->tmp_a.alloc(5 * n * sizeof(Fr)));
    TRY(P->eval_partial.alloc((size_t)kMaxEval * pk_eval_max_blocks(nq) * sizeof(Fr)));
    if (!P->eval_out.ptr) {
      TRY(P->eval_out.alloc(kMaxEval * sizeof(Fr),
                            hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable));
      PLK_HIP_TRY(hipHostGetDevicePointer(&P->eval_dev, P->eval_out.ptr, 0));
    }
    // 4 nq: the four wires' 12 coset blocks transform in one batch (24n of scratch: the output
    // doubles as the other ping-pong buffer, ntt_run_batch)
    TRY(P->ntt_scratch.alloc(4 * nq * sizeof(Fr)));
    Fr* nsc = P->ntt_scratch.as<Fr>();

    // transcript seeded like Prover::new (prover.rs:54-55): Transcript::base(label, vk, m)
    Transcript tr(key->label);
    {
      const char dom[] = "circuit_size";
      tr.append_message("dom-sep", reinterpret_cast<const uint8_t*>(dom), sizeof(dom) - 1);
      tr.append_u64("n", m);
      const char* labels[15] = {"q_m", "q_l", "q_r", "q_o", "q_c", "q_4", "q_arith", "q_range",
                                "q_logic", "q_fixed_group_add", "q_variable_group_add",
                                "s_sigma_1", "s_sigma_2", "s_sigma_3", "s_sigma_4"};
      for (int i = 0; i < 15; ++i) tr.append_commitment(labels[i], key->comms[i]);
    }
    // public inputs (prover.rs:90-105)
    std::vector<std::pair<uint64_t, Fr>> pis;
    for (uint64_t i = 0; i < m; ++i)
      if (cs->gates[i].code & kPiBit) pis.emplace_back(i, gate_unpack(cs, i).pi);
    for (auto& p : pis) tr.append_scalar("pi", p.second);
    if (pi_count) *pi_count = pis.size();
    if (public_inputs)
      for (size_t i = 0; i < pis.size() && i < pi_cap; ++i) public_inputs[i] = fr_to(pis[i].second);

    // ---- round 1: wires -> idft -> blind(1) -> commit (prover.rs:107-158)
    {  // witness upload through pinned staging, in chunks: the CPU copy of chunk i+1
       // overlaps the DMA of chunk i (the previous proof's DMA finished at its last wait)
      const size_t bytes = cs->witness.size() * sizeof(Fr);
      TRY(P->pin_witness.alloc(bytes));
      const size_t chunk = 8u << 20;
      const char* src = reinterpret_cast<const char*>(cs->witness.data());
      char* pin = P->pin_witness.as<char>();
      char* dst = P->witness.as<char>();
      for (size_t off = 0; off < bytes; off += chunk) {
        const size_t len = std::min(chunk, bytes - off);
        std::memcpy(pin + off, src + off, len);
        PLK_HIP_TRY(hipMemcpyAsync(dst + off, pin + off, len, hipMemcpyHostToDevice, s));
      }
    }
    Fr* wl = P->wires_lag.as<Fr>();
    Fr* wc = P->wires_coef.as<Fr>();
    TRY(pk_gather_wires(P->witness.as<Fr>(), key->wire_idx.as<uint32_t>(), m, n, wl, s));
    {  // the four wire idfts as one batch (one launch per pass instead of four)
      NttBatch b;
      b.in_stride = n;
      b.out_stride = S;
      TRY(ntt_run_batch(key->dom, wl, wc, n, -1, 0, nsc, s, 4, b));
    }
    BlindBatch bb{};
    bb.npoly = 4;
    for (int c = 0; c < 4; ++c) {
      bb.poly[c] = wc + c * S;  // blind(1): b(X)(X^n - 1), two scalars per wire, drawn in order
      bb.b[c].count = 2;
      bb.b[c].r[0] = rng.fr();
      bb.b[c].r[1] = rng.fr();
    }
    TRY(pk_blind_batch(bb, n, s));
    plk_g1 wcom[4];
    TRY(prover_commit(P, {wc, wc + S, wc + 2 * S, wc + 3 * S}, {n + 2, n + 2, n + 2, n + 2}, wcom,
                      nullptr));
    tr.append_commitment("a_w", wcom[0]);
    tr.append_commitment("b_w", wcom[1]);
    tr.append_commitment("c_w", wcom[2]);
    tr.append_commitment("d_w", wcom[3]);

    // ---- round 2: permutation grand product z (prover.rs:160-199)
    const Fr beta = tr.challenge_scalar("beta");
    tr.append_scalar("beta", beta);
    const Fr gamma = tr.challenge_scalar("gamma");
    Fr* num = P->num.as<Fr>();
    Fr* den = P->den.as<Fr>();
    TRY(pk_perm_numden(wl, key->sigma_lag.as<Fr>(), key->dom->tw_fwd.as<Fr>(), n, beta, gamma, K1,
                       K2, K3, num, den, s));
    Fr* st = P->scan_tmp.as<Fr>();
    TRY(pk_scan(num, num, n, true, false, true, st, s));   // N_i = prod_{j<i} num_j
    TRY(pk_scan(den, den, n, true, true, false, st, s));   // S_i = prod_{j>=i} den_j
    const uint64_t nb = pk_scan_tmp_elems(n) - 1;
    const Fr dtot = d2h_fr(st + nb, s);                    // prod of all den_j
    TRY(pk_mul3(num, den, fe_inv(dtot), P->z_lag.as<Fr>(), n, s));
    Fr* zc = P->z_coef.as<Fr>();
    TRY(ntt_run(key->dom, P->z_lag.as<Fr>(), zc, n, -1, 0, nsc, s, 1));
    {
      BlindArgs b{};
      b.count = 3;
      for (int i = 0; i < 3; ++i) b.r[i] = rng.fr();
      TRY(pk_blind(zc, n, b, s));
    }
    plk_g1 zcom;
    TRY(prover_commit(P, {zc}, {n + 3}, &zcom, nullptr));
    tr.append_commitment("z", zcom);

    // ---- round 3: quotient (prover.rs:201-287, quotient_poly.rs)
    const Fr alpha = tr.challenge_scalar("alpha");
    const Fr range_sep = tr.challenge_scalar("range separation challenge");
    const Fr logic_sep = tr.challenge_scalar("logic separation challenge");
    const Fr fixed_sep = tr.challenge_scalar("fixed base separation challenge");
    const Fr var_sep = tr.challenge_scalar("variable base separation challenge");
    Fr* pil = P->pi_lag.as<Fr>();
    // pin_small: the PI values uploaded here (sized once: queued copies keep pointing into it)
    TRY(P->pin_small.alloc(std::max<size_t>(pis.size(), 1) * sizeof(Fr)));
    // PI(X) = idft of the public-input vector (prover.rs:229): for a few public inputs
    // straight from its definition, one product per input and coefficient (no upload, no
    // transform); otherwise the vector is uploaded and transformed
    const bool pi_direct = !pis.empty() && pis.size() <= (size_t)kPiDirect;
    if (pi_direct) {
      PiDirect pd{};
      pd.count = (uint32_t)pis.size();
      for (size_t i = 0; i < pis.size(); ++i) {
        pd.idx[i] = pis[i].first;
        pd.c[i] = fe_mul(pis[i].second, key->dom->n_inv);
      }
      TRY(pk_pi_coef(pd, key->dom->tw_inv.as<Fr>(), n, P->pi_coef.as<Fr>(), s));
    } else if (!pis.empty()) {
      PLK_HIP_TRY(hipMemsetAsync(pil, 0, n * sizeof(Fr), s));
      for (size_t i = 0; i < pis.size(); ++i) {
        P->pin_small.as<Fr>()[i] = pis[i].second;
        PLK_HIP_TRY(hipMemcpyAsync(pil + pis[i].first, P->pin_small.as<Fr>() + i, sizeof(Fr),
                                   hipMemcpyHostToDevice, s));
      }
    }
    // the six polynomials over the quotient domain (quotient_poly.rs:54-58,145 over g H_8n
    // there): each a batch of the three coset blocks (prover.hpp) in one launch per pass
    Fr* ev = P->evq.as<Fr>();  // z, a, b, c, d, pi, nq points each
    auto coset_fwd = [&](const Fr* in, Fr* out, uint64_t len, const DevBuf& table) {
      NttBatch b;
      b.in_stride = 0;
      b.out_stride = n2;
      b.pre = table.as<Fr>();
      b.pre_stride = n + 8;
      return ntt_run_batch(key->domq, in, out, len, 1, 1, nsc, s, kQBlocks, b);
    };
    if (!pis.empty() && !pi_direct)
      TRY(ntt_run(key->dom, pil, P->pi_coef.as<Fr>(), n, -1, 0, nsc, s, 1));
    TRY(coset_fwd(zc, ev + 0 * nq, n + 3, key->coset_s));
    // wire evaluations at exponent -1 and PI at +1 for k_quotient's redundant-form
    // arithmetic (QuotientArgs): scaled coset tables, no extra pass
    {  // the four wires' coset blocks as ONE batch of 12 (NttBatch::group: wire c, block m)
      NttBatch b;
      b.group = kQBlocks;
      b.in_stride = 0;
      b.in_group_stride = S;
      b.out_stride = n2;
      b.pre = key->coset_w.as<Fr>();
      b.pre_stride = n + 8;
      TRY(ntt_run_batch(key->domq, wc, ev + nq, n + 2, 1, 1, nsc, s, 4 * kQBlocks, b));
    }
    // PI(X) over the coset; a circuit without public inputs has PI = 0 (the term is skipped)
    if (!pis.empty()) TRY(coset_fwd(P->pi_coef.as<Fr>(), ev + 5 * nq, n, key->coset_pi));
    const Fr alpha2 = fe_sqr(alpha);
    QuotientArgs qa{};
    qa.z = ev;
    qa.a = ev + nq;
    qa.b = ev + 2 * nq;
    qa.c = ev + 3 * nq;
    qa.d = ev + 4 * nq;
    qa.pi = pis.empty() ? nullptr : ev + 5 * nq;
    qa.l1 = key->l1q.as<Fr>();
    qa.alpha2 = alpha2;
    qa.sel = key->selq.as<Fr>();
    qa.sigma = key->sigmaq.as<Fr>();
    qa.elements = key->domq->tw_fwd.as<Fr>();
    qa.out = P->quotq.as<Fr>();
    qa.nq = nq;
    qa.log_blk = key->k + 1;
    qa.g = key->domq->g;
    qa.alpha = alpha;
    qa.beta = beta;
    qa.gamma = gamma;
    qa.k1 = K1;
    qa.k2 = K2;
    qa.k3 = K3;
    qa.range_sep = range_sep;
    qa.kappa = fe_sqr(range_sep);
    qa.kappa2 = fe_sqr(qa.kappa);
    qa.kappa3 = fe_mul(qa.kappa2, qa.kappa);
    qa.has_range = key->has_range ? 1 : 0;
    qa.logic_sep = logic_sep;
    qa.lk = fe_sqr(logic_sep);
    qa.lk2 = fe_sqr(qa.lk);
    qa.lk3 = fe_mul(qa.lk2, qa.lk);
    qa.lk4 = fe_mul(qa.lk3, qa.lk);
    qa.has_logic = key->has_logic ? 1 : 0;
    qa.fixed_sep = fixed_sep;
    qa.fk = fe_sqr(fixed_sep);
    qa.fk2 = fe_sqr(qa.fk);
    qa.fk3 = fe_mul(qa.fk2, qa.fk);
    qa.var_sep = var_sep;
    qa.vk = fe_sqr(var_sep);
    qa.vk2 = fe_sqr(qa.vk);
    qa.edwards_d = edwards_d();
    qa.has_fixed = key->has_fixed ? 1 : 0;
    qa.has_var = key->has_var ? 1 : 0;
    for (int j = 0; j < 2 * kQBlocks; ++j) qa.vh_inv[j] = key->vh_inv[j];
    {  // exponent-scaled constants for k_quotient (x[e] = x R 2^(-5e); [-1] = R' domain)
      auto em1 = [](const Fr& x) { return fe_to_rx_domain(x); };
      auto em2 = [](const Fr& x) { return fe_to_rx_domain(fe_to_rx_domain(x)); };
      const Fr one = fe_one<FrCfg>(), two = fe_dbl(one);
      for (int mb = 0; mb < kQBlocks; ++mb) qa.rx_bg[mb] = em2(fe_mul(beta, key->s_m[mb]));
      qa.rx_beta = em2(beta);
      qa.rx_gamma = em1(gamma);
      qa.rx_one_w = em1(one);
      qa.rx_two_w = em1(two);
      qa.rx_three_w = em1(fe_add(two, one));
      qa.rx_kappa = em1(qa.kappa);
      qa.rx_kappa2 = em1(qa.kappa2);
      qa.rx_kappa3 = em1(qa.kappa3);
      qa.rx_alpha2 = em1(alpha2);
      for (int j = 0; j < 2 * kQBlocks; ++j) qa.rx_vh[j] = em2(key->vh_inv[j]);
      qa.rx_32 = fr_u64(32);
      qa.rx_inv32 = fe_inv(qa.rx_32);
    }
    TRY(pk_quotient(qa, s));
    Fr* tc = P->t_coef.as<Fr>();
    {  // t = coset_idft over the quotient domain (quotient_poly.rs:115): the three blocks'
       // inverse transforms (post-scaled by (2n)^-1 3^-1 s_m^-k) in place, then the radix-3
       // combine into the 6n coefficients (t has at most 4n + 7; the rest are zero)
      NttBatch b;
      b.in_stride = b.out_stride = n2;
      b.post = key->icoset_q.as<Fr>();
      b.post_stride = n2;
      TRY(ntt_run_batch(key->domq, P->quotq.as<Fr>(), P->quotq.as<Fr>(), n2, -1, 1, nsc, s,
                        kQBlocks, b));
      TRY(pk_coset3_combine(P->quotq.as<Fr>(), n2, key->comb, tc, s));
    }
    // split into t_low, t_mid, t_high (n each) and t_4 = t[3n..] (prover.rs:252-265)
    plk_g1 tcom[4];
    // t_4 is t[3n..8n) in the reference (prover.rs:259) and t[3n..6n) here. For a satisfied
    // circuit t has degree <= 4n + 6 on either domain (prover.hpp), so t_4 ends below n + 8:
    // committing at most n + 8 points changes no commitment, and the zero check of the rest
    // fails for an unsatisfied circuit (its interpolant does not vanish there) where the
    // reference's commit fails (t_4 past the trimmed SRS, prover.rs:262-265) — including
    // tiny circuits whose trimmed SRS covers all of t[3n..6n)
    TRY(prover_commit(P, {tc, tc + n, tc + 2 * n, tc + 3 * n}, {n, n, n, nq - 3 * n}, tcom,
                      nullptr, n + 8));
    // its commit succeeded, so everything past the committed prefix is zero: t and t_4 end at
    // 3n + t4_len for the evaluation and the opening below
    const uint64_t t4_len = std::min<uint64_t>(
        n + 8, std::min<uint64_t>(key->srs->n, key->n_trim));
    tr.append_commitment("t_low", tcom[0]);
    tr.append_commitment("t_mid", tcom[1]);
    tr.append_commitment("t_high", tcom[2]);
    tr.append_commitment("t_4", tcom[3]);

    // ---- round 4 / 5: evaluations and linearization (linearization_poly.rs:22-134)
    const Fr zeta = tr.challenge_scalar("z_challenge");
    const Fr zw = fe_mul(zeta, key->dom->omega);
    const Fr* qc = key->q_coef.as<Fr>();
    const Fr* sc = key->sigma_coef.as<Fr>();
    // r(X) = sum_t s_t p_t(X) (arithmetic / range / logic / curve widgets' linearize and the
    // permutation's): its polynomials p_t are known now, its scalars s_t only from the
    // evaluations. So r is never formed: its terms' values at z join the batch of the 16
    // proof evaluations (one launch, one read-back), r(z) = sum_t s_t p_t(z) is taken on the
    // host — the same field element — and the opening aggregate carries v s_t p_t itself.
    struct RTerm {
      const Fr* p;
      uint64_t len;
      int ev;  // index of p(z) in the evaluation batch
    };
    std::vector<RTerm> rt;
    EvalBatch eb{};
    const Fr* polys[16] = {tc, wc, wc + S, wc + 2 * S, wc + 3 * S, sc, sc + n, sc + 2 * n,
                           qc + QARITH * n, qc + QC * n, qc + QL * n, qc + QR * n,
                           wc, wc + S, wc + 3 * S, zc};
    const uint64_t lens[16] = {3 * n + t4_len, n + 2, n + 2, n + 2, n + 2, n, n, n, n, n, n, n,
                               n + 2, n + 2, n + 2, n + 3};
    uint32_t ne = 0;
    for (int i = 0; i < 16; ++i, ++ne) {
      eb.poly[i] = polys[i];
      eb.len[i] = lens[i];
      eb.x[i] = i < 12 ? zeta : zw;
    }
    auto rterm = [&](const Fr* p, uint64_t len, int have) {
      if (have < 0) {  // a new evaluation at z
        eb.poly[ne] = p;
        eb.len[ne] = len;
        eb.x[ne] = zeta;
        have = (int)ne++;
      }
      rt.push_back(RTerm{p, len, have});
    };
    // in the order the scalars are formed below
    rterm(qc + QM * n, n, -1);
    rterm(qc + QL * n, n, 10);
    rterm(qc + QR * n, n, 11);
    rterm(qc + QO * n, n, -1);
    rterm(qc + Q4 * n, n, -1);
    rterm(qc + QC * n, n, 9);
    if (key->has_range) rterm(qc + QRANGE * n, n, -1);
    if (key->has_logic) rterm(qc + QLOGIC * n, n, -1);
    if (key->has_fixed) rterm(qc + QFIXED * n, n, -1);
    if (key->has_var) rterm(qc + QVAR * n, n, -1);
    rterm(zc, n + 3, -1);
    rterm(sc + 3 * n, n, -1);
    // the evaluations land in host memory (no copy dispatch): read once the stream is done
    TRY(pk_eval(eb, ne, 3 * n + t4_len, P->eval_partial.as<Fr>(), static_cast<Fr*>(P->eval_dev), s));
    Fr evs[kMaxEval];
    PLK_HIP_TRY(stream_wait(s));
    std::memcpy(evs, P->eval_out.ptr, ne * sizeof(Fr));
    const Fr t_eval = evs[0], a_e = evs[1], b_e = evs[2], c_e = evs[3], d_e = evs[4];
    const Fr s1_e = evs[5], s2_e = evs[6], s3_e = evs[7];
    const Fr qar_e = evs[8], qc_e = evs[9], ql_e = evs[10], qr_e = evs[11];
    const Fr an_e = evs[12], bn_e = evs[13], dn_e = evs[14], perm_e = evs[15];
    // the scalars s_t of r(X) = arithmetic::linearize + range::linearize + ... + permutation
    std::vector<Fr> rs;
    rs.push_back(fe_mul(qar_e, fe_mul(a_e, b_e)));  // q_m
    rs.push_back(fe_mul(qar_e, a_e));               // q_l
    rs.push_back(fe_mul(qar_e, b_e));               // q_r
    rs.push_back(fe_mul(qar_e, c_e));               // q_o
    rs.push_back(fe_mul(qar_e, d_e));               // q_4
    rs.push_back(qar_e);                            // q_c
    if (key->has_range) {
      const Fr two = fe_dbl(one), three = fe_add(two, one);
      auto delta = [&](const Fr& f) {
        return fe_mul(fe_mul(f, fe_sub(f, one)), fe_mul(fe_sub(f, two), fe_sub(f, three)));
      };
      auto four = [](const Fr& v) { return fe_dbl(fe_dbl(v)); };
      Fr r = delta(fe_sub(c_e, four(d_e)));
      r = fe_add(r, fe_mul(delta(fe_sub(b_e, four(c_e))), qa.kappa));
      r = fe_add(r, fe_mul(delta(fe_sub(a_e, four(b_e))), qa.kappa2));
      r = fe_add(r, fe_mul(delta(fe_sub(dn_e, four(a_e))), qa.kappa3));
      rs.push_back(fe_mul(r, range_sep));
    }
    if (key->has_logic) {  // logic::linearize: q_logic(X) * sep * (...) at the evaluations
      const Fr two = fe_dbl(one), three = fe_add(two, one), four = fe_dbl(two);
      auto delta = [&](const Fr& f) {
        return fe_mul(fe_mul(f, fe_sub(f, one)), fe_mul(fe_sub(f, two), fe_sub(f, three)));
      };
      const Fr qa_ = fe_sub(an_e, fe_mul(four, a_e));
      const Fr qb_ = fe_sub(bn_e, fe_mul(four, b_e));
      const Fr qd_ = fe_sub(dn_e, fe_mul(four, d_e));
      Fr r = delta(qa_);
      r = fe_add(r, fe_mul(delta(qb_), qa.lk));
      r = fe_add(r, fe_mul(delta(qd_), qa.lk2));
      r = fe_add(r, fe_mul(fe_sub(c_e, fe_mul(qa_, qb_)), qa.lk3));
      r = fe_add(r, fe_mul(logic_xor_and(qa_, qb_, c_e, qd_, qc_e), qa.lk4));
      rs.push_back(fe_mul(r, logic_sep));
    }
    if (key->has_fixed) {  // curve_scalar::linearize at the evaluations (q_l/q_r/q_c evals)
      const Fr w = widget_fixed_base(a_e, an_e, b_e, bn_e, c_e, d_e, dn_e, ql_e, qr_e, qc_e,
                                     qa.fk, qa.fk2, qa.fk3, qa.edwards_d);
      rs.push_back(fe_mul(w, fixed_sep));
    }
    if (key->has_var) {  // curve_addtion::linearize
      const Fr w = widget_var_base(a_e, an_e, b_e, bn_e, c_e, d_e, dn_e, qa.vk, qa.vk2,
                                   qa.edwards_d);
      rs.push_back(fe_mul(w, var_sep));
    }
    // z(X) * [(a + b z + g)(b + b K1 z + g)(c + b K2 z + g)(d + b K3 z + g) alpha + L1(z) alpha^2]
    const Fr bz = fe_mul(beta, zeta);
    Fr idc = fe_mul(fe_add(fe_add(a_e, bz), gamma), fe_add(fe_add(b_e, fe_mul(K1, bz)), gamma));
    idc = fe_mul(idc, fe_add(fe_add(c_e, fe_mul(K2, bz)), gamma));
    idc = fe_mul(idc, fe_add(fe_add(d_e, fe_mul(K3, bz)), gamma));
    idc = fe_mul(idc, alpha);
    const Fr zh = fe_sub(fe_pow_u64(zeta, n), one);  // Z_H(z)
    const Fr l1 = fe_mul(zh, fe_inv(fe_mul(fr_u64(n), fe_sub(zeta, one))));
    rs.push_back(fe_add(idc, fe_mul(l1, alpha2)));
    // -sigma_4(X) * (a + b s1 + g)(b + b s2 + g)(c + b s3 + g) beta perm_eval alpha
    Fr cpc = fe_add(fe_add(a_e, fe_mul(beta, s1_e)), gamma);
    cpc = fe_mul(cpc, fe_add(fe_add(b_e, fe_mul(beta, s2_e)), gamma));
    cpc = fe_mul(cpc, fe_add(fe_add(c_e, fe_mul(beta, s3_e)), gamma));
    cpc = fe_mul(fe_mul(cpc, fe_mul(beta, perm_e)), alpha);
    rs.push_back(fe_neg(cpc));
    if (rs.size() != rt.size()) return PLK_E_DEVICE;  // the two lists are built in one order
    Fr r_e = fe_zero<FrCfg>();  // r(z) = sum_t s_t p_t(z)
    for (size_t t = 0; t < rt.size(); ++t) r_e = fe_add(r_e, fe_mul(rs[t], evs[rt[t].ev]));

    const char* elabels[17] = {"a_eval", "b_eval", "c_eval", "d_eval", "a_next_eval",
                               "b_next_eval", "d_next_eval", "s_sigma_1_eval", "s_sigma_2_eval",
                               "s_sigma_3_eval", "q_arith_eval", "q_c_eval", "q_l_eval",
                               "q_r_eval", "perm_eval", "t_eval", "r_eval"};
    const Fr evals17[17] = {a_e, b_e, c_e, d_e, an_e, bn_e, dn_e, s1_e, s2_e, s3_e,
                            qar_e, qc_e, ql_e, qr_e, perm_e, t_eval, r_e};
    for (int i = 0; i < 17; ++i) tr.append_scalar(elabels[i], evals17[i]);

    // ---- openings (prover.rs:407-452): both v challenges precede both commits
    const Fr v1 = tr.challenge_scalar("v_challenge");
    const Fr v2 = tr.challenge_scalar("v_challenge");
    const Fr zn = fe_pow_u64(zeta, n), z2n = fe_sqr(zn), z3n = fe_mul(z2n, zn);
    // W(X) = (sum v1^i p_i(X)) / (X - z), p = [quot, r, a, b, c, d, s1, s2, s3]
    // with quot = t_low + z^n t_mid + z^2n t_high + z^3n t_4 and r = sum_t s_t p_t expanded
    // in place (scalars v1 s_t)
    LinComb la{};
    auto lt = [&](const Fr* p, uint64_t len, const Fr& sc_) {
      la.p[la.terms] = p;
      la.len[la.terms] = len;
      la.s[la.terms] = sc_;
      ++la.terms;
    };
    if (4 + rt.size() + 7 > (size_t)kMaxTerms) return PLK_E_DEVICE;
    // the aggregate and its quotient by (X - z) stop where t_4 does (same polynomials,
    // same commits)
    const uint64_t agg_len = std::max<uint64_t>(n + 3, t4_len);
    lt(tc, n, one);
    lt(tc + n, n, zn);
    lt(tc + 2 * n, n, z2n);
    lt(tc + 3 * n, t4_len, z3n);
    Fr vp = v1;
    for (size_t t = 0; t < rt.size(); ++t) lt(rt[t].p, rt[t].len, fe_mul(vp, rs[t]));
    for (int c = 0; c < 4; ++c) {
      vp = fe_mul(vp, v1);
      lt(wc + c * S, n + 2, vp);
    }
    for (int c = 0; c < 3; ++c) {
      vp = fe_mul(vp, v1);
      lt(sc + c * n, n, vp);
    }
    Fr* ag = P->agg.as<Fr>();
    TRY(pk_lincomb(la, ag, agg_len, s));
    Fr* w1 = P->w_coef.as<Fr>();
    Fr* w2 = w1 + 5 * n;
    TRY(pk_ruffini(ag, agg_len, zeta, w1, P->tmp_a.as<Fr>(), st, s));
    // W'(X) = (z + v2 a + v2^2 b + v2^3 d) / (X - z w)
    LinComb lb{};
    lb.terms = 4;
    lb.p[0] = zc;
    lb.len[0] = n + 3;
    lb.s[0] = one;
    lb.p[1] = wc;
    lb.len[1] = n + 2;
    lb.s[1] = v2;
    lb.p[2] = wc + S;
    lb.len[2] = n + 2;
    lb.s[2] = fe_sqr(v2);
    lb.p[3] = wc + 3 * S;
    lb.len[3] = n + 2;
    lb.s[3] = fe_mul(lb.s[2], v2);
    Fr* ag2 = P->agg2.as<Fr>();
    TRY(pk_lincomb(lb, ag2, n + 3, s));
    TRY(pk_ruffini(ag2, n + 3, zw, w2, P->tmp_a.as<Fr>(), st, s));
    plk_g1 wcm[2];
    TRY(prover_commit(P, {w1, w2}, {agg_len - 1, n + 2}, wcm, nullptr));

    // ---- proof (proof.rs:36-66)
    proof->a_comm = wcom[0];
    proof->b_comm = wcom[1];
    proof->c_comm = wcom[2];
    proof->d_comm = wcom[3];
    proof->z_comm = zcom;
    proof->t_low_comm = tcom[0];
    proof->t_mid_comm = tcom[1];
    proof->t_high_comm = tcom[2];
    proof->t_4_comm = tcom[3];
    proof->w_z_chall_comm = wcm[0];
    proof->w_z_chall_w_comm = wcm[1];
    proof->a_eval = fr_to(a_e);
    proof->b_eval = fr_to(b_e);
    proof->c_eval = fr_to(c_e);
    proof->d_eval = fr_to(d_e);
    proof->a_next_eval = fr_to(an_e);
    proof->b_next_eval = fr_to(bn_e);
    proof->d_next_eval = fr_to(dn_e);
    proof->q_arith_eval = fr_to(qar_e);
    proof->q_c_eval = fr_to(qc_e);
    proof->q_l_eval = fr_to(ql_e);
    proof->q_r_eval = fr_to(qr_e);
    proof->s_sigma_1_eval = fr_to(s1_e);
    proof->s_sigma_2_eval = fr_to(s2_e);
    proof->s_sigma_3_eval = fr_to(s3_e);
    proof->r_poly_eval = fr_to(r_e);
    proof->perm_eval = fr_to(perm_e);
    return PLK_OK;
  } catch (const std::bad_alloc&) {
    return PLK_E_OOM;
  } catch (...) {
    return PLK_E_DEVICE;
  }
}

}  // extern "C"

plk_prover::~plk_prover() {
  if (own_stream && stream) (void)hipStreamDestroy(stream);
  plk::msm_workspace_delete(ws);
}

plk_key::~plk_key() = default;
