// Host-side helpers of the predict path (no GPU work).
//
// mmpfn_siphash24_rows: the fingerprint feature's row hash (reference model/preprocessing.py:476-479,
// Python `hash(row.tobytes())`, reproducible only under PYTHONHASHSEED=0 -- CPython 3.10's bytes hash
// is SipHash-2-4 keyed by the hash secret, all zero under that seed).  The reference hashes every
// member's test rows once per predict; in numpy the per-word rounds over a few hundred rows are
// overhead-bound (~1 ms per member), this is one pass over the bytes.
#include <cstdint>
#include <cstring>

#include "../../include/mmpfn_hip.h"

namespace {

inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

inline void sipround(uint64_t& v0, uint64_t& v1, uint64_t& v2, uint64_t& v3) {
  v0 += v1;
  v1 = rotl(v1, 13) ^ v0;
  v0 = rotl(v0, 32);
  v2 += v3;
  v3 = rotl(v3, 16) ^ v2;
  v0 += v3;
  v3 = rotl(v3, 21) ^ v0;
  v2 += v1;
  v1 = rotl(v1, 17) ^ v2;
  v2 = rotl(v2, 32);
}

int64_t siphash24_zero_key(const unsigned char* p, int64_t nb) {
  if (nb == 0) return 0;  // hash(b"") == 0
  uint64_t v0 = 0x736F6D6570736575ull, v1 = 0x646F72616E646F6Dull, v2 = 0x6C7967656E657261ull,
           v3 = 0x7465646279746573ull;
  const int64_t nw = nb / 8;
  for (int64_t j = 0; j < nw; ++j) {
    uint64_t m;
    std::memcpy(&m, p + 8 * j, 8);  // little endian
    v3 ^= m;
    sipround(v0, v1, v2, v3);
    sipround(v0, v1, v2, v3);
    v0 ^= m;
  }
  uint64_t last = (uint64_t)(nb & 0xFF) << 56;
  for (int64_t k = 0; k < nb - 8 * nw; ++k) last |= (uint64_t)p[8 * nw + k] << (8 * k);
  v3 ^= last;
  sipround(v0, v1, v2, v3);
  sipround(v0, v1, v2, v3);
  v0 ^= last;
  v2 ^= 0xFF;
  for (int i = 0; i < 4; ++i) sipround(v0, v1, v2, v3);
  const int64_t h = (int64_t)(v0 ^ v1 ^ v2 ^ v3);
  return h == -1 ? -2 : h;  // CPython reserves -1
}

}  // namespace

extern "C" int mmpfn_siphash24_rows(const void* rows, int64_t n_rows, int64_t row_bytes, int64_t* out) {
  if (n_rows < 0 || row_bytes < 0 || (n_rows > 0 && (!out || (row_bytes > 0 && !rows)))) return MMPFN_ERR_INVALID;
  const unsigned char* b = (const unsigned char*)rows;
  for (int64_t i = 0; i < n_rows; ++i) out[i] = siphash24_zero_key(b + i * row_bytes, row_bytes);
  return MMPFN_OK;
}
