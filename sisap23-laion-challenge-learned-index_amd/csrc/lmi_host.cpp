// Host utilities of the drop-in (no GPU work): a multi-threaded content hash
// of a host buffer.
//
// li.LearnedIndex keeps the bucket-sorted corpus in HBM between calls, where
// the reference re-gathers every bucket from the DataFrame on every call
// (LearnedIndex.py:152-153, :168).  A cached index may only be served for
// byte-identical inputs, so a call that cannot trust the frame's identity
// (LearnedIndex.attach) hashes its bytes.  15 GB of fp16 clip768 at 10M: the
// python xxh3 binding holds the GIL (one core, ~6.6 GB/s, ~2.3 s); this hash
// runs the blocks on OpenMP threads and is memory-bound.
//
// The hash: the buffer is cut into 4-MiB blocks; each block is hashed with
// four independent 64-bit lanes of xxh64-style rounds over 32-byte stripes
// (tail bytes folded one by one), and the block hashes are combined in block
// order, so the value does not depend on the thread count.  Not
// cryptographic: it detects changed data, not adversarial collisions.
#include <cstdint>
#include <cstring>
#include <vector>

#include <omp.h>

#include "../../include/lmi_hip.h"

namespace {

constexpr uint64_t P1 = 0x9E3779B185EBCA87ull;
constexpr uint64_t P2 = 0xC2B2AE3D27D4EB4Full;
constexpr uint64_t P3 = 0x165667B19E3779F9ull;
constexpr uint64_t P5 = 0x27D4EB2F165667C5ull;
constexpr uint64_t kBlock = 4ull << 20;

inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t round1(uint64_t acc, uint64_t w) { return rotl(acc + w * P2, 31) * P1; }
inline uint64_t avalanche(uint64_t h) {
    h ^= h >> 33;
    h *= P2;
    h ^= h >> 29;
    h *= P3;
    h ^= h >> 32;
    return h;
}

uint64_t hash_block(const unsigned char* p, uint64_t n, uint64_t seed) {
    uint64_t a0 = seed + P1 + P2, a1 = seed + P2, a2 = seed, a3 = seed - P1;
    uint64_t i = 0;
    for (; i + 32 <= n; i += 32) {
        uint64_t w[4];
        std::memcpy(w, p + i, 32);
        a0 = round1(a0, w[0]);
        a1 = round1(a1, w[1]);
        a2 = round1(a2, w[2]);
        a3 = round1(a3, w[3]);
    }
    uint64_t h = rotl(a0, 1) + rotl(a1, 7) + rotl(a2, 12) + rotl(a3, 18) + n;
    for (; i < n; ++i) h = rotl(h ^ (p[i] * P5), 11) * P1;
    return avalanche(h);
}

}  // namespace

extern "C" uint64_t lmi_host_hash64(const void* data, uint64_t n_bytes, int32_t threads) {
    const unsigned char* p = static_cast<const unsigned char*>(data);
    if (p == nullptr || n_bytes == 0) return avalanche(n_bytes + P5);
    const uint64_t nb = (n_bytes + kBlock - 1) / kBlock;
    std::vector<uint64_t> hb(nb);
    const int nt = threads > 0 ? threads : omp_get_max_threads();
#pragma omp parallel for schedule(static) num_threads(nt)
    for (int64_t b = 0; b < (int64_t)nb; ++b) {
        const uint64_t off = (uint64_t)b * kBlock;
        const uint64_t len = n_bytes - off < kBlock ? n_bytes - off : kBlock;
        hb[b] = hash_block(p + off, len, (uint64_t)b);
    }
    uint64_t h = n_bytes * P5;
    for (uint64_t b = 0; b < nb; ++b) h = round1(h, hb[b]);
    return avalanche(h);
}
