// sg_device.h -- device-side arithmetic that must match the reference bit for bit.
// Compiled with -ffp-contract=off: every f32 op below rounds once (no FMA),
// as Rust's f32 ops do in graph/mod.rs:328.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace sg {

// ---------------------------------------------------------------------------
// Packed lexicographic path key.
// PathProperties (graph/mod.rs:297-313) orders by latency, then packet loss.
// Loss is a non-negative f32 in [0, 1] whose bit pattern (<= 0x3F800000 < 2^30)
// is order-preserving, so key = (latency << 30) | bits(loss) compares like
// PathProperties as one u64 while latency < 2^34 - 1 (17.2 s).  Latency
// saturates at LAT_SAT; any saturated key marks "overflow or unreachable" and
// the row falls back to the wide (u64 latency + f32 loss) kernel.
// ---------------------------------------------------------------------------
constexpr int LOSS_BITS = 30;
constexpr uint64_t LOSS_MASK = (1ull << LOSS_BITS) - 1;
constexpr uint64_t LAT_SAT = (1ull << (64 - LOSS_BITS)) - 1;  // 2^34 - 1
constexpr uint64_t KEY_INF = ~0ull;                            // (LAT_SAT << 30) | LOSS_MASK

__host__ __device__ __forceinline__ uint64_t key_lat(uint64_t k) { return k >> LOSS_BITS; }
__host__ __device__ __forceinline__ uint32_t key_loss_bits(uint64_t k) {
  return (uint32_t)(k & LOSS_MASK);
}

// PathProperties::add (graph/mod.rs:322-331) with the edge's (1f32 - loss)
// precomputed: loss' = 1f32 - (1f32 - a) * (1f32 - e).  The subtraction
// 1f32 - e is a single rounded op in both places, so precomputing it is exact.
__device__ __forceinline__ float fold_loss(float a, float one_minus_e) {
  float oma = __fsub_rn(1.0f, a);
  float prod = __fmul_rn(oma, one_minus_e);
  return __fsub_rn(1.0f, prod);
}

// key(u) + edge, latency saturating at LAT_SAT.  edge_lat is pre-clamped to
// LAT_SAT on upload, so the u64 sum cannot wrap.
__device__ __forceinline__ uint64_t relax_key(uint64_t ku, uint64_t edge_lat, float edge_om) {
  uint64_t lat = key_lat(ku) + edge_lat;
  lat = lat < LAT_SAT ? lat : LAT_SAT;
  float loss = fold_loss(__uint_as_float(key_loss_bits(ku)), edge_om);
  return (lat << LOSS_BITS) | (uint64_t)__float_as_uint(loss);
}

// ---------------------------------------------------------------------------
// RNG: rand_xoshiro 0.7.0 Xoshiro256PlusPlus + SplitMix64 seed_from_u64
// (host/host.rs:221), rand 0.9 StandardUniform<f64> = (x >> 11) * 2^-53
// (worker.rs:360).
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint64_t rotl64(uint64_t x, int k) {
  return (x << k) | (x >> (64 - k));
}

__host__ __device__ __forceinline__ uint64_t splitmix64_next(uint64_t& st) {
  st += 0x9E3779B97F4A7C15ull;
  uint64_t z = st;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Xoshiro {
  uint64_t s0, s1, s2, s3;
  __host__ __device__ __forceinline__ uint64_t next_u64() {
    uint64_t r = rotl64(s0 + s3, 23) + s0;
    uint64_t t = s1 << 17;
    s2 ^= s0;
    s3 ^= s1;
    s1 ^= s2;
    s0 ^= s3;
    s2 ^= t;
    s3 = rotl64(s3, 45);
    return r;
  }
  __host__ __device__ __forceinline__ double next_f64() {
    return (double)(next_u64() >> 11) * (1.0 / 9007199254740992.0);
  }
};

__host__ __device__ inline Xoshiro xoshiro_seed_from_u64(uint64_t seed) {
  Xoshiro x;
  uint64_t st = seed;
  x.s0 = splitmix64_next(st);
  x.s1 = splitmix64_next(st);
  x.s2 = splitmix64_next(st);
  x.s3 = splitmix64_next(st);
  if ((x.s0 | x.s1 | x.s2 | x.s3) == 0) {  // from_seed's all-zero guard
    st = 0;
    x.s0 = splitmix64_next(st);
    x.s1 = splitmix64_next(st);
    x.s2 = splitmix64_next(st);
    x.s3 = splitmix64_next(st);
  }
  return x;
}

}  // namespace sg
