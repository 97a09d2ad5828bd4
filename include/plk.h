/*
 * plk.h — C ABI of the MI355X PLONK hot path (BLS12-381 Fr NTT family + G1 MSM/KZG commit).
 *
 * This is the drop-in boundary. In the reference the path sits behind Rust generic
 * structs of un-vendored crates (no FFI exists there); each entry point
 * below replaces one of those calls. The host-side mirror that calls this ABI with the
 * reference's names is dusk-plonk_amd/plonk.py + dusk-plonk_amd/prover.py (Python, used by
 * the tests and bench.py); the C++ prover behind plk_prove is dusk-plonk_amd/csrc/prover.hip.
 * INTEGRATION.md shows the Rust-side binding.
 *
 * Conventions
 *  - plk_fr is BlsScalar exactly as the reference stores it: 4 little-endian u64 limbs
 *    in Montgomery form with R = 2^256 (pinned by /root/reference/src/lib.rs:583-588).
 *  - plk_g1 is G1Affine: x, y as 6 LE u64 limbs of Montgomery Fp (R = 2^384), plus an
 *    infinity flag (0/1) widened to u64. Outputs are canonical (fully reduced, and the
 *    point at infinity is written as x = y = 0, infinity = 1).
 *  - Host pointers are caller-owned; in-place use (same in/out) is allowed.
 *    Entry points with the _dev suffix take device pointers and a hipStream_t (passed as
 *    void*, NULL = the context's stream) and are stream-ordered.
 *  - Every entry point returns a plk_status; nothing throws or aborts across the ABI.
 *  - One plk_ctx per GPU. A context may be used from one thread at a time; concurrent
 *    streams must pass their own scratch buffers (plk_ntt_dev) / workspaces.
 */
#ifndef PLK_H
#define PLK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PLK_ABI_VERSION 2

typedef struct { uint64_t l[4]; } plk_fr;                          /* 32 bytes  */
typedef struct { uint64_t x[6]; uint64_t y[6]; uint64_t infinity; } plk_g1; /* 104 bytes */

typedef enum {
  PLK_OK = 0,
  PLK_E_DEGREE = 1,   /* commit: polynomial (trailing zeros stripped) longer than the SRS
                         — zksnarks PlonkParams::commit error path (prover.rs:133-452) */
  PLK_E_ARG = 2,      /* bad argument (null pointer, length > domain, bad log_n, ...) */
  PLK_E_DEVICE = 3,   /* HIP runtime error */
  PLK_E_OOM = 4,      /* device allocation failed */
  PLK_E_NODEV = 5,    /* no GPU visible / HIP unavailable */
  PLK_E_UNSUPPORTED = 6 /* reserved: a feature this backend does not implement */
} plk_status;

typedef struct plk_ctx plk_ctx;
typedef struct plk_domain plk_domain;
typedef struct plk_srs plk_srs;
typedef struct plk_composer plk_composer;
typedef struct plk_key plk_key;

/* ---- library / context ------------------------------------------------------------- */
int plk_abi_version(void);
const char* plk_status_str(int status);
/* Build provenance (no reference counterpart): "src=<16 hex> flags=<16 hex> variant=<name>",
 * src = a hash of csrc/ *.hip, csrc/ *.hpp and this header as they were compiled, flags = a hash
 * of the hipcc flags (build_ext.py source_id / flags_id). The Python mirror refuses a library
 * whose src differs from the tree it is loaded from (plonk.check_build). */
const char* plk_build_info(void);
/* Number of visible GPUs (0 when no GPU; never fails for lack of one). */
int plk_device_count(int* out);
int plk_ctx_create(int device, plk_ctx** out);
int plk_ctx_destroy(plk_ctx* ctx);
/* The context's default stream (hipStream_t) — for callers that chain _dev calls. */
int plk_ctx_stream(plk_ctx* ctx, void** stream_out);
int plk_ctx_synchronize(plk_ctx* ctx);

/* ---- evaluation domains: poly_commit::Fft<Fr> -------------------------------------- */
/* Fft::new(k) (prover.rs:88, quotient_poly.rs:52, key.rs:83,222). Cached per ctx and k:
 * w = ROOT_OF_UNITY^(2^(32-k)), coset shift g = 7, tables resident in HBM. 0 <= k <= 27. */
int plk_domain_get(plk_ctx* ctx, uint32_t log_n, plk_domain** out);
/* Fft::size(), generator() (= w), generator_inv(), size_inv(), and the coset shift g, g^-1.
 * Any output pointer may be NULL. (prover.rs:252,446; key.rs:205-207) */
int plk_domain_info(const plk_domain* d, uint64_t* size, plk_fr* generator,
                    plk_fr* generator_inv, plk_fr* size_inv, plk_fr* coset, plk_fr* coset_inv);
/* Fft.elements: out[i] = w^i, i < n (permutation.rs:148,246). */
int plk_domain_elements(const plk_domain* d, plk_fr* out);
/* Fft::compute_vanishing_poly_over_coset(poly_degree) (key.rs:291):
 * out[i] = (g * w^i)^poly_degree - 1, i < n. */
int plk_domain_vanishing_over_coset(const plk_domain* d, uint64_t poly_degree, plk_fr* out);

/* ---- the NTT family (host buffers) --------------------------------------------------
 * dir = +1: Fft::dft (coset = 0) / Fft::coset_dft (coset = 1)
 *           input: len_in <= n coefficients (zero-padded to n); output: n evaluations.
 *           (permutation.rs:232; quotient_poly.rs:54-58,145,237; key.rs:226-245)
 * dir = -1: Fft::idft (coset = 0) / Fft::coset_idft (coset = 1)
 *           input: len_in <= n evaluations (zero-padded); output: n coefficients.
 *           (prover.rs:121-124,192,229; quotient_poly.rs:115,271; permutation.rs:194-197;
 *            key.rs:121-131)
 * `inout` must hold n elements; natural order in and out. */
int plk_ntt(plk_domain* d, plk_fr* inout, size_t len_in, int dir, int coset);
/* plk_ntt on the caller's stream (hipStream_t as void*, NULL = the context's stream), the
 * signature of SURVEY §8b: same semantics, host buffer in and out, returns once `inout`
 * holds the result (the reference's Fft calls block). Staging and scratch are stream-ordered
 * allocations of its own, so callers on different streams may share one domain. */
int plk_ntt_stream(plk_domain* d, plk_fr* inout, size_t len_in, int dir, int coset, void* stream);
/* Device-pointer variant: d_in -> d_out (may alias; both hold n elements). d_scratch is
 * NULL (use the domain's scratch — then calls on one domain must share one stream) or a
 * device buffer of 2*n elements owned by the caller. */
int plk_ntt_dev(plk_domain* d, const plk_fr* d_in, plk_fr* d_out, size_t len_in, int dir,
                int coset, plk_fr* d_scratch, void* stream);
/* Batched device variant: `count` independent vectors, vector v at d_inout + v*n. */
int plk_ntt_batch_dev(plk_domain* d, plk_fr* d_inout, size_t count, int dir, int coset,
                      void* stream);

/* ---- SRS and KZG commit: zksnarks::plonk::PlonkParams<TatePairing> ------------------ */
/* PlonkParams::setup(k, rng) restated with an explicit secret tau (Montgomery Fr):
 * g1[i] = [tau^i]G1 for i < n_points, generated on the GPU. If out_points != NULL the
 * points are also copied to the host. The returned SRS is resident and MSM-ready. */
int plk_srs_setup(plk_ctx* ctx, const plk_fr* tau, size_t n_points, plk_g1* out_points,
                  plk_srs** out);
/* The slice [start, start + n_points) of the same SRS (g1[i] = [tau^i]G1 for i in the
 * range): the per-GPU shard of a sharded MSM. */
int plk_srs_setup_range(plk_ctx* ctx, const plk_fr* tau, uint64_t start, size_t n_points,
                        plk_g1* out_points, plk_srs** out);
/* Load an existing SRS (e.g. a trimmed PlonkParams) from host affine points. */
int plk_srs_load(plk_ctx* ctx, const plk_g1* points, size_t n_points, plk_srs** out);
int plk_srs_destroy(plk_srs* srs);
int plk_srs_len(const plk_srs* srs, size_t* n_points);
/* Copy SRS points [start, start+count) back to the host. */
int plk_srs_points(const plk_srs* srs, size_t start, size_t count, plk_g1* out);

/* Raw MSM: out = sum_{i<len} scalars[i] * g1[i], len <= n_points (msm_curve_addition,
 * proof.rs:507; the inner loop of commit). */
int plk_msm(plk_srs* srs, const plk_fr* scalars, size_t len, plk_g1* out);
/* PlonkParams::commit(&Coefficients) (prover.rs:133-136,194,262-265,440,452;
 * key.rs:138-159): strips trailing zeros; PLK_E_DEGREE if the rest is longer than the
 * SRS; otherwise out = MSM over the SRS prefix. */
int plk_commit(plk_srs* srs, const plk_fr* coeffs, size_t len, plk_g1* out);
/* Device-pointer commit (coefficients already in HBM, e.g. straight from plk_ntt_dev). */
int plk_commit_dev(plk_srs* srs, const plk_fr* d_coeffs, size_t len, plk_g1* out,
                   void* stream);

/* Batched device commit: `count` independent polynomials (d_coeffs[k], lens[k]) committed
 * as one GPU batch (their kernels share launches; the latency-bound reduction tails of the
 * batch overlap). Used for the prover's independent commit groups: the 4 wire commits
 * (prover.rs:133-136), the 4 quotient chunks (:262-265) and the 2 openings (:440,452).
 * statuses (nullable) gets each commit's status; returns PLK_E_DEGREE if any failed. */
int plk_commit_batch_dev(plk_srs* srs, const plk_fr* const* d_coeffs, const size_t* lens,
                         size_t count, plk_g1* outs, int* statuses, void* stream);

/* Bucket-range part of plk_commit_batch_dev (round 5; SURVEY §8e, the north star's "partial
 * bucket sums for a single large MSM"): the same commits, but only the Pippenger buckets of
 * part `part` of `parts` (parts a power of two): bucket range [part, part + 1) x 2^(c-1) /
 * parts of the SRS's window size c. outs[k] is that range's share sum_{b in range} (b + 1) S_b
 * of commit k; the shares of parts 0 .. parts-1 sum (plk_g1_sum) to plk_commit_batch_dev's
 * outputs. Every part reads all scalars and the whole window table, sorts and accumulates
 * only its buckets' entries and reduces only its buckets: one GPU per part, each doing
 * ~1/parts of the accumulation AND of the bucket reduction (the SRS-slice split,
 * plk_prover_shard / plk_msm_sharded, divides only the accumulation). The degree check runs
 * in every part (same status everywhere). PLK_E_ARG unless 2^(c-1) > 32768 (a wide bucket
 * set, c >= 17: SRS >= 2^16 points) and 2^(c-1) / parts >= 2^14. */
int plk_commit_batch_dev_part(plk_srs* srs, const plk_fr* const* d_coeffs, const size_t* lens,
                              size_t count, uint32_t part, uint32_t parts, plk_g1* outs,
                              int* statuses, void* stream);

/* PlonkParams::compute_aggregate_witness(&[p_0..p_(k-1)], &point, &v) (prover.rs:422-438,
 * 444-450): W(X) = (sum_i v^i p_i(X)) / (X - point), the remainder dropped (Ruffini). The
 * k polynomials (d_polys[i], lens[i] coefficients) are device pointers; d_out receives
 * *out_len = max(lens) - 1 coefficients (0 when every polynomial is constant or empty),
 * stream-ordered. point and v must be canonical (PLK_E_ARG otherwise). The same division
 * plk_prove runs for its two openings; exported so the primitive itself can be replaced. */
int plk_aggregate_witness_dev(plk_ctx* ctx, const plk_fr* const* d_polys, const size_t* lens,
                              size_t count, const plk_fr* point, const plk_fr* v,
                              plk_fr* d_out, size_t* out_len, void* stream);
/* Host-buffer variant on the context's stream; returns when `out` holds the result. */
int plk_aggregate_witness(plk_ctx* ctx, const plk_fr* const* polys, const size_t* lens,
                          size_t count, const plk_fr* point, const plk_fr* v, plk_fr* out,
                          size_t* out_len);

/* Host-side sum of n affine points (canonical affine out): the local fold after the RCCL
 * all-gather of per-GPU partial commitments of a sharded MSM. Needs no GPU. */
int plk_g1_sum(const plk_g1* points, size_t n, plk_g1* out);

/* One large MSM split over the GPUs of a node from ONE process:
 * per_gpu[i] holds the SRS points following those of per_gpu[0..i-1] (e.g.
 * plk_srs_setup_range on consecutive ranges, one slice per device). Each slice's MSM of its
 * scalar slice runs concurrently (one host thread per slice, each on its own device and
 * stream) and the partial points are folded on the host (plk_g1_sum):
 * out = sum_{i<len} scalars[i] * g1[i], len <= total points. The multi-process form (one
 * rank per GPU, RCCL all-gather of the partials) is dusk-plonk_amd/parallel.py. */
int plk_msm_sharded(plk_srs* const* per_gpu, int n_gpu, const plk_fr* scalars, size_t len,
                    plk_g1* out);

/* ---- instrumentation (bench / profiling) ------------------------------------------- */
/* Milliseconds of the dominant kernel of the most recent plk_commit/plk_msm on this SRS
 * (bucket accumulation), measured with HIP events on the launching stream; and the
 * number of bucket-accumulation point additions it performed. */
int plk_srs_last_msm_stats(const plk_srs* srs, float* accumulate_ms, uint64_t* point_adds,
                           uint32_t* window_bits);
/* Cumulative accumulation statistics since the last reset (measurement only): summed
 * k_accumulate time (HIP events on the MSM's stream), launches, point additions and MSM
 * points (scalar counts over all slots). */
int plk_srs_msm_stats_reset(plk_srs* srs);
int plk_srs_cum_msm_stats(const plk_srs* srs, double* accumulate_ms, uint64_t* launches,
                          uint64_t* point_adds, uint64_t* points);

/* ---- prover: Plonk composer, PlonkKey::compile, Prover::create_proof --------------------
 * The callers of the hot path, restated on the C++ host with every O(n) step
 * on the GPU. A constraint is one width-4 gate
 *   q_m a b + q_l a + q_r b + q_o o + q_4 d + q_c + PI = 0   (src/lib.rs:546) plus the
 * widget selectors; a, b, o, d are witness indices. Field order follows
 * zksnarks::Constraint. */
typedef struct {
  plk_fr q_m, q_l, q_r, q_o, q_4, q_c, q_arith, q_range, q_logic, q_fixed_group_add,
      q_variable_group_add;
  uint32_t a, b, o, d;
  uint32_t has_public, _pad;
  plk_fr public_input;
} plk_constraint;

/* zksnarks Proof (src/prover/proof.rs:36-66) with ProofEvaluations in construction order
 * (src/prover/linearization_poly.rs:117-134). */
typedef struct {
  plk_g1 a_comm, b_comm, c_comm, d_comm, z_comm, t_low_comm, t_mid_comm, t_high_comm, t_4_comm,
      w_z_chall_comm, w_z_chall_w_comm;
  plk_fr a_eval, b_eval, c_eval, d_eval, a_next_eval, b_next_eval, d_next_eval, q_arith_eval,
      q_c_eval, q_l_eval, q_r_eval, s_sigma_1_eval, s_sigma_2_eval, s_sigma_3_eval, r_poly_eval,
      perm_eval;
} plk_proof;

/* Plonk::initialize (src/lib.rs:121-134): zero/one witnesses, their constant gates and
 * two rounds of dummy gates. */
int plk_composer_create(plk_composer** out);
int plk_composer_destroy(plk_composer* c);
int plk_composer_size(const plk_composer* c, size_t* gates, size_t* witnesses);
int plk_composer_append_witness(plk_composer* c, const plk_fr* value, uint32_t* wire);
int plk_composer_witness_value(const plk_composer* c, uint32_t wire, plk_fr* value);
int plk_composer_set_witness(plk_composer* c, uint32_t wire, const plk_fr* value);
/* append_public (lib.rs:708-719) */
int plk_composer_append_public(plk_composer* c, const plk_fr* value, uint32_t* wire);
/* append_gate (lib.rs:546-550, q_arith = 1) / append_custom_gate (lib.rs:224-240) */
int plk_composer_append_gate(plk_composer* c, const plk_constraint* s);
int plk_composer_append_custom_gate(plk_composer* c, const plk_constraint* s);
/* gate_add / gate_mul (lib.rs:1169-1197): q_o = -1, output evaluated and appended */
int plk_composer_gate_eval(plk_composer* c, const plk_constraint* s, uint32_t* out_wire);
int plk_composer_assert_equal(plk_composer* c, uint32_t a, uint32_t b);            /* :721 */
int plk_composer_assert_equal_constant(plk_composer* c, uint32_t a, const plk_fr* constant,
                                       const plk_fr* public_input /* nullable */);  /* :766 */
int plk_composer_component_boolean(plk_composer* c, uint32_t a);                   /* :859 */
/* component_range (lib.rs:1066-1163): constrain `a` to num_bits (<= 256) bits with the
 * range widget; an out-of-range value makes create_proof fail (tests/range.rs:82-84). */
int plk_composer_component_range(plk_composer* c, uint32_t a, size_t num_bits);
/* The bench circuit: `gates` chained gates x' = x*y + x (q_m = q_l = 1, q_o = -1). */
int plk_composer_synthetic_chain(plk_composer* c, size_t gates, uint64_t seed);
/* Plonk::instance(): public inputs sorted by gate index, and their indexes. */
int plk_composer_public_inputs(const plk_composer* c, plk_fr* values, uint64_t* indexes,
                               size_t cap, size_t* count);
/* The circuit as the composer holds it (Plonk::constraints and the witness vector,
 * lib.rs:103-115): gates[i] for i < min(cap, m) and witness[j] for j < min(wcap, #witness);
 * *m / *nw receive the full sizes. For external checkers and serialisation. */
int plk_composer_export(const plk_composer* c, plk_constraint* gates, size_t cap,
                        plk_fr* witness, size_t wcap, size_t* m, size_t* nw);

/* PlonkKey::compile_with_circuit (src/key.rs:63-327): device-resident proving key for the
 * circuit's structure, committed against `srs` (trimmed to next_pow2(m + 6) + 8 points).
 * All five widgets are proven: arithmetic, range, logic, fixed-base scalar multiplication
 * and variable-base addition (quotient_poly.rs:128-262, linearization_poly.rs:136-225). */
int plk_key_compile(plk_srs* srs, const plk_composer* circuit, const char* label, plk_key** out);
int plk_key_destroy(plk_key* key);
/* n (padded domain), m (gates) and the 15 verifier-key commitments in transcript order
 * q_m q_l q_r q_o q_c q_4 q_arith q_range q_logic q_fixed_group_add q_variable_group_add
 * s_sigma_1..4. */
int plk_key_info(const plk_key* key, uint64_t* n, uint64_t* m, plk_g1* commitments);
/* Prover::create_proof (src/prover.rs:67-474) for a circuit with the key's structure and
 * its own witness values. Blinding randomness comes from `seed` (SplitMix64). Fails with
 * PLK_E_DEGREE exactly where the reference's commit fails for an unsatisfied circuit, and
 * with PLK_E_ARG when the circuit's structure (gates, wires, selectors, public-input
 * positions) differs from the one the key was compiled from or its witness vector is too
 * short for the key's wires. */
int plk_prove(plk_key* key, const plk_composer* circuit, uint64_t seed, plk_proof* proof,
              plk_fr* public_inputs, size_t pi_cap, size_t* pi_count);

/* ---- prover lanes: several proofs in flight over one key ----------------------------
 * Prover: Clone + create_proof(&self) may run concurrently in the reference.
 * A plk_prover is one such concurrent prover: its own HIP stream, MSM workspace, NTT
 * scratch and per-proof buffers, sharing the key's device-resident tables and the SRS
 * window table read-only (one copy per GPU however many proofs are in flight). Provers of
 * one key may run plk_prover_prove from different threads at the same time. Destroy every
 * prover of a key before the key. plk_prove(key, ...) is plk_prover_prove on a default
 * prover the key owns (on the context's stream); it is thread-safe, but concurrent
 * plk_prove calls on one key are serialised on that prover — use plk_prover_create for
 * proofs in parallel. */
typedef struct plk_prover plk_prover;
int plk_prover_create(plk_key* key, plk_prover** out);
int plk_prover_destroy(plk_prover* p);
/* The prover's stream (hipStream_t). */
int plk_prover_stream(plk_prover* p, void** stream_out);
/* Prover::create_proof (prover.rs:67-474) on this prover; arguments as plk_prove. */
int plk_prover_prove(plk_prover* p, const plk_composer* circuit, uint64_t seed, plk_proof* proof,
                     plk_fr* public_inputs, size_t pi_cap, size_t* pi_count);
/* k_accumulate statistics of this prover's MSMs (see plk_srs_cum_msm_stats); reset != 0
 * clears the cumulative figures after reading them. Any output may be NULL. */
int plk_prover_msm_stats(plk_prover* p, int reset, double* accumulate_ms, uint64_t* launches,
                         uint64_t* point_adds, uint64_t* points);

/* ---- sharded commits: one proof, its MSMs split over the GPUs of a node ------------------
 * BASELINE configs[4] / SURVEY §8e. One process (rank) per GPU proves the SAME circuit with
 * the same seed; every rank runs the NTT / elementwise rounds on its own GPU (replicas, they
 * are a minority of the proof) and each commit — the 4 wire commits (prover.rs:133-136),
 * z (:194), the 4 quotient chunks (:262-265) and the 2 openings (:440,452) — is split by
 * SRS index: rank r runs the Pippenger over its slice [slice_start, slice_start +
 * slice_len) of every polynomial against `slice` (plk_srs_setup_range on the same tau), then
 * the ranks exchange their partial points (13 words + a status word per commit) with ONE
 * all-gather per commit group and each folds them on the host (plk_g1_sum order: rank 0
 * first). Proofs are byte-identical to the unsharded plk_prove on any rank.
 * The all-gather is the caller's (RCCL over xGMI under torch.distributed in
 * dusk-plonk_amd/parallel.py): `allgather(user, send, bytes, recv)` must place every rank's
 * `bytes` of `send` at recv + rank * bytes and return 0 (non-zero: PLK_E_DEVICE). Slices
 * must tile [0, N) in rank order with N >= the key's trimmed SRS; every rank calls
 * plk_prover_prove for every proof, in the same order (the exchange is a collective).
 * world = 1 with a slice and an all-gather runs the same exchange path with one rank (the
 * sharded code path on one GPU); world = 1 with slice = allgather = NULL is unsharded. */
typedef int (*plk_allgather_fn)(void* user, const void* send, size_t bytes, void* recv);
int plk_prover_shard(plk_prover* p, plk_srs* slice, uint64_t slice_start, int rank, int world,
                     plk_allgather_fn allgather, void* user);
/* The same sharded proof with each commit split by BUCKET RANGE instead of SRS slice (round 6;
 * the north star's "partial bucket sums"): every rank keeps the key's whole SRS and window
 * table and runs every commit of the group over all of its points, sorting, accumulating and
 * reducing only bucket range `rank` of `world` (plk_commit_batch_dev_part's split, so each rank
 * also does 1/world of the bucket reduction, which the slice split repeats on every rank); the
 * shares go through the same all-gather and fold, so proofs are byte-identical. PLK_E_ARG
 * unless `world` is a power of two and the key's SRS has a wide bucket set with >= 2^14
 * buckets per part (c >= 17: SRS >= 2^16 points; c = 20 from 2^20 points: world <= 32) — the
 * caller then keeps plk_prover_shard's slices. Undone by plk_prover_shard. */
int plk_prover_shard_buckets(plk_prover* p, int rank, int world, plk_allgather_fn allgather,
                             void* user);

/* ---- Proof wire format (SCALE, src/prover/proof.rs:11,36) ---------------------------------
 * The reference derives parity-scale-codec Encode/Decode for Proof: fields in declaration
 * order, 11 Commitment<G1Affine> then ProofEvaluations. The element encodings live in the
 * un-vendored bls-12-381 / zksnarks crates; ASSUMED here (parity unpinned): G1Affine as its
 * fields x, y (Fq = [u64; 6] Montgomery limbs, LE) and is_infinity (bool, 1 byte) = 97 B;
 * Fr as [u64; 4] Montgomery limbs, LE = 32 B; ProofEvaluations in plk_proof order. Total
 * PLK_PROOF_SCALE_BYTES. Decode rejects (PLK_E_ARG) a wrong length, a non-boolean flag,
 * limbs >= the modulus, and finite points not on y^2 = x^3 + 4. The identity (ASSUMED
 * encoding) is written as x = 0, y = 0, is_infinity = 1; decode takes is_infinity = 1 with
 * (x, y) = (0, 0) or zkcrypto's (0, one) as the identity and returns it as (0, 0, 1); other
 * coordinates under the flag are rejected. DELIBERATE DIVERGENCE (parity unpinned): a
 * derived SCALE Decode plus zkcrypto's flag-only is_identity would accept ANY (x, y) under
 * is_infinity = 1 as the identity; this decoder is strict so that one proof has one byte
 * string (a verifier hashing proof bytes sees no malleable identity encodings). No fixture
 * in the reference covers either behaviour. */
#define PLK_PROOF_SCALE_BYTES (11 * 97 + 16 * 32)
int plk_proof_encode(const plk_proof* proof, uint8_t* out, size_t cap, size_t* len);
int plk_proof_decode(const uint8_t* in, size_t len, plk_proof* proof);

/* ---- test support ---------------------------------------------------------------- */
/* Elementwise device field arithmetic on host arrays (used by the parity tests to pin the
 * gfx950 multiplier against the oracle): field 0 = Fr (4 limbs), 1 = Fp (6 limbs);
 * op 0 = a*b, 1 = a+b, 2 = a-b, 3 = a^2, 4 = a^-1 (Montgomery form in and out). */
int plk_debug_field_op(plk_ctx* ctx, int field, int op, const uint64_t* a, const uint64_t* b,
                       uint64_t* out, size_t n);

#ifdef __cplusplus
}
#endif
#endif /* PLK_H */
