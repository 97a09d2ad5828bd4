/*
 * plk.h — C ABI of the MI355X PLONK hot path (BLS12-381 Fr NTT family + G1 MSM/KZG commit).
 *
 * This is the drop-in boundary. In the reference the path sits behind Rust generic
 * structs of un-vendored crates (no FFI exists there); each entry point
 * below replaces one of those calls. The host-side mirror that calls this ABI with the
 * reference's names is dusk-plonk_amd/plonk.py (Python, used by the tests) and
 * dusk-plonk_amd/csrc/plonk.hpp (C++). INTEGRATION.md shows the Rust-side binding.
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

#define PLK_ABI_VERSION 1

typedef struct { uint64_t l[4]; } plk_fr;                          /* 32 bytes  */
typedef struct { uint64_t x[6]; uint64_t y[6]; uint64_t infinity; } plk_g1; /* 104 bytes */

typedef enum {
  PLK_OK = 0,
  PLK_E_DEGREE = 1,   /* commit: polynomial (trailing zeros stripped) longer than the SRS
                         — zksnarks PlonkParams::commit error path (prover.rs:133-452) */
  PLK_E_ARG = 2,      /* bad argument (null pointer, length > domain, bad log_n, ...) */
  PLK_E_DEVICE = 3,   /* HIP runtime error */
  PLK_E_OOM = 4,      /* device allocation failed */
  PLK_E_NODEV = 5     /* no GPU visible / HIP unavailable */
} plk_status;

typedef struct plk_ctx plk_ctx;
typedef struct plk_domain plk_domain;
typedef struct plk_srs plk_srs;

/* ---- library / context ------------------------------------------------------------- */
int plk_abi_version(void);
const char* plk_status_str(int status);
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

/* Host-side sum of n affine points (canonical affine out): the local fold after the RCCL
 * all-gather of per-GPU partial commitments of a sharded MSM. Needs no GPU. */
int plk_g1_sum(const plk_g1* points, size_t n, plk_g1* out);

/* ---- instrumentation (bench / profiling) ------------------------------------------- */
/* Milliseconds of the dominant kernel of the most recent plk_commit/plk_msm on this SRS
 * (bucket accumulation), measured with HIP events on the launching stream; and the
 * number of bucket-accumulation point additions it performed. */
int plk_srs_last_msm_stats(const plk_srs* srs, float* accumulate_ms, uint64_t* point_adds,
                           uint32_t* window_bits);

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
