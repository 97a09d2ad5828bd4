// transcript.hpp — merlin transcript (STROBE-128 / Keccak-f[1600]) for the prover's host
// side: dusk-plonk's Transcript / TranscriptProtocol (zksnarks, un-vendored; used at
// /root/reference/src/prover.rs:54-55,99-452). Host-only; a few hundred bytes per proof.
// Pinned by merlin's published vector (tests/test_transcript.py).
#pragma once
#include <cstdint>
#include <cstring>
#include <string>

#include "ff.hpp"
#include "g1.hpp"

namespace plk {

class Keccak {
 public:
  static void f1600(uint8_t* st) {
    static const uint64_t RC[24] = {
        0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
        0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
        0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
        0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
        0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
        0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
    static const int ROT[5][5] = {{0, 36, 3, 41, 18}, {1, 44, 10, 45, 2}, {62, 6, 43, 15, 61},
                                  {28, 55, 25, 21, 56}, {27, 20, 39, 8, 14}};
    uint64_t A[5][5], B[5][5], C[5], D[5];
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y) std::memcpy(&A[x][y], st + 8 * (x + 5 * y), 8);
    for (int r = 0; r < 24; ++r) {
      for (int x = 0; x < 5; ++x) C[x] = A[x][0] ^ A[x][1] ^ A[x][2] ^ A[x][3] ^ A[x][4];
      for (int x = 0; x < 5; ++x) D[x] = C[(x + 4) % 5] ^ rol(C[(x + 1) % 5], 1);
      for (int x = 0; x < 5; ++x)
        for (int y = 0; y < 5; ++y) A[x][y] ^= D[x];
      for (int x = 0; x < 5; ++x)
        for (int y = 0; y < 5; ++y) B[y][(2 * x + 3 * y) % 5] = rol(A[x][y], ROT[x][y]);
      for (int x = 0; x < 5; ++x)
        for (int y = 0; y < 5; ++y) A[x][y] = B[x][y] ^ (~B[(x + 1) % 5][y] & B[(x + 2) % 5][y]);
      A[0][0] ^= RC[r];
    }
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y) std::memcpy(st + 8 * (x + 5 * y), &A[x][y], 8);
  }

 private:
  static uint64_t rol(uint64_t x, int n) { return n ? (x << n) | (x >> (64 - n)) : x; }
};

class Strobe128 {
 public:
  explicit Strobe128(const std::string& label) {
    std::memset(st_, 0, sizeof st_);
    const uint8_t init[6] = {1, kR + 2, 1, 0, 1, 96};
    std::memcpy(st_, init, 6);
    std::memcpy(st_ + 6, "STROBEv1.0.2", 12);
    Keccak::f1600(st_);
    meta_ad(reinterpret_cast<const uint8_t*>(label.data()), label.size(), false);
  }
  void meta_ad(const uint8_t* d, size_t n, bool more) {
    begin_op(kM | kA, more);
    absorb(d, n);
  }
  void ad(const uint8_t* d, size_t n, bool more) {
    begin_op(kA, more);
    absorb(d, n);
  }
  void prf(uint8_t* out, size_t n, bool more) {
    begin_op(kI | kA | kC, more);
    for (size_t i = 0; i < n; ++i) {
      out[i] = st_[pos_];
      st_[pos_] = 0;
      if (++pos_ == kR) run_f();
    }
  }

 private:
  static constexpr uint8_t kI = 1, kA = 2, kC = 4, kT = 8, kM = 16, kK = 32;
  static constexpr uint8_t kR = 166;
  uint8_t st_[200];
  uint8_t pos_ = 0, pos_begin_ = 0, cur_flags_ = 0;

  void run_f() {
    st_[pos_] ^= pos_begin_;
    st_[pos_ + 1] ^= 0x04;
    st_[kR + 1] ^= 0x80;
    Keccak::f1600(st_);
    pos_ = 0;
    pos_begin_ = 0;
  }
  void absorb(const uint8_t* d, size_t n) {
    for (size_t i = 0; i < n; ++i) {
      st_[pos_] ^= d[i];
      if (++pos_ == kR) run_f();
    }
  }
  void begin_op(uint8_t flags, bool more) {
    if (more) return;  // continuation of the same operation (flags checked by callers)
    const uint8_t old_begin = pos_begin_;
    pos_begin_ = pos_ + 1;
    cur_flags_ = flags;
    const uint8_t hdr[2] = {old_begin, flags};
    absorb(hdr, 2);
    if ((flags & (kC | kK)) && pos_ != 0) run_f();
  }
};

class Transcript {
 public:
  explicit Transcript(const std::string& label) : s_("Merlin v1.0") {
    append_message("dom-sep", reinterpret_cast<const uint8_t*>(label.data()), label.size());
  }
  void append_message(const char* label, const uint8_t* msg, size_t n) {
    s_.meta_ad(reinterpret_cast<const uint8_t*>(label), std::strlen(label), false);
    const uint32_t len = (uint32_t)n;
    uint8_t le[4] = {(uint8_t)len, (uint8_t)(len >> 8), (uint8_t)(len >> 16), (uint8_t)(len >> 24)};
    s_.meta_ad(le, 4, true);
    s_.ad(msg, n, false);
  }
  void append_u64(const char* label, uint64_t x) {
    uint8_t b[8];
    for (int i = 0; i < 8; ++i) b[i] = (uint8_t)(x >> (8 * i));
    append_message(label, b, 8);
  }
  void challenge_bytes(const char* label, uint8_t* out, size_t n) {
    s_.meta_ad(reinterpret_cast<const uint8_t*>(label), std::strlen(label), false);
    const uint32_t len = (uint32_t)n;
    uint8_t le[4] = {(uint8_t)len, (uint8_t)(len >> 8), (uint8_t)(len >> 16), (uint8_t)(len >> 24)};
    s_.meta_ad(le, 4, true);
    s_.prf(out, n, false);
  }

  // ---- TranscriptProtocol (dusk-plonk) -----------------------------------------------
  // append_scalar: 32 bytes, little-endian canonical
  void append_scalar(const char* label, const Fr& s_mont) {
    const Fr c = fe_from_mont(s_mont);
    uint8_t b[32];
    for (int i = 0; i < 8; ++i)
      for (int k = 0; k < 4; ++k) b[4 * i + k] = (uint8_t)(c.v[i] >> (8 * k));
    append_message(label, b, 32);
  }
  // append_commitment: zkcrypto-format compressed G1 (48 bytes, big-endian x with the
  // compression / infinity / sort flags in the top bits of byte 0)
  void append_commitment(const char* label, const plk_g1& p) {
    uint8_t b[48];
    g1_compress(p, b);
    append_message(label, b, 48);
  }
  // challenge_scalar: Fr::from_bytes_wide(64 challenge bytes), Montgomery form out
  Fr challenge_scalar(const char* label) {
    uint8_t b[64];
    challenge_bytes(label, b, 64);
    return fr_from_bytes_wide(b);
  }

  static Fr fr_from_bytes_wide(const uint8_t* b) {
    // (lo + hi * 2^256) mod r: lo*R^2 and hi*R^3 in Montgomery form (R = 2^256)
    Fr lo, hi;
    for (int i = 0; i < 8; ++i) {
      lo.v[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) |
                ((uint32_t)b[4 * i + 3] << 24);
      hi.v[i] = (uint32_t)b[32 + 4 * i] | ((uint32_t)b[33 + 4 * i] << 8) |
                ((uint32_t)b[34 + 4 * i] << 16) | ((uint32_t)b[35 + 4 * i] << 24);
    }
    // the spare-bit Montgomery multiply needs canonical inputs: 2^256 < 3r, so at most
    // two conditional subtractions bring each half below r
    for (int k = 0; k < 2; ++k) {
      fe_reduce_once(lo);
      fe_reduce_once(hi);
    }
    Fr r2;
    for (int i = 0; i < 8; ++i) r2.v[i] = FrCfg::R2[i];
    const Fr r3 = fe_mul(r2, r2);  // R^2 * R^2 / R = R^3
    return fe_add(fe_mul(lo, r2), fe_mul(hi, r3));
  }

  static void g1_compress(const plk_g1& p, uint8_t* out) {
    std::memset(out, 0, 48);
    if (p.infinity) {
      out[0] = 0xc0;
      return;
    }
    Fp x, y;
    for (int k = 0; k < 6; ++k) {
      x.v[2 * k] = (uint32_t)p.x[k];
      x.v[2 * k + 1] = (uint32_t)(p.x[k] >> 32);
      y.v[2 * k] = (uint32_t)p.y[k];
      y.v[2 * k + 1] = (uint32_t)(p.y[k] >> 32);
    }
    x = fe_from_mont(x);
    y = fe_from_mont(y);
    for (int i = 0; i < 12; ++i)
      for (int k = 0; k < 4; ++k) out[47 - (4 * i + k)] = (uint8_t)(x.v[i] >> (8 * k));
    // sort flag: y > (p-1)/2  <=>  2y > p - 1  <=>  y != 0 and y is the larger root
    const Fp ny = fe_neg(y);
    bool larger = false;
    for (int i = 11; i >= 0; --i) {
      if (y.v[i] != ny.v[i]) {
        larger = y.v[i] > ny.v[i];
        break;
      }
    }
    out[0] |= 0x80 | (larger ? 0x20 : 0);
  }

 private:
  Strobe128 s_;
};

}  // namespace plk
