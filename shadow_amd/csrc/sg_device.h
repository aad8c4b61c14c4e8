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
// Loss is a non-negative f32 in [0, 1], whose bit pattern is order-preserving,
// so key = (latency u32 << 32) | bits(loss) compares like PathProperties as one
// u64, and one 64-bit store is an untorn (latency, loss) update.  Latency adds
// saturate at LAT32_SAT (v_add_u32 clamp); a key whose latency reached
// LAT32_SAT means "overflow or unreachable" and its row is redone by the wide
// (u64 latency + f32 loss) kernel.  KEY_INF = (LAT32_SAT, loss 1.0) is a fixed
// point of relax32: sat(LAT32_SAT + l) = LAT32_SAT and 1 - (1 - 1) * om = 1.
// ---------------------------------------------------------------------------
constexpr uint32_t LAT32_SAT = 0xFFFFFFFFu;
constexpr uint64_t KEY_INF = 0xFFFFFFFF3F800000ull;

__host__ __device__ __forceinline__ uint32_t key_lat(uint64_t k) { return (uint32_t)(k >> 32); }
__host__ __device__ __forceinline__ uint32_t key_loss_bits(uint64_t k) { return (uint32_t)k; }

// PathProperties::add (graph/mod.rs:322-331) with the edge's (1f32 - loss)
// precomputed: loss' = 1f32 - (1f32 - a) * (1f32 - e).  The subtraction
// 1f32 - e is a single rounded op in both places, so precomputing it is exact.
__device__ __forceinline__ float fold_loss(float a, float one_minus_e) {
  float oma = __fsub_rn(1.0f, a);
  float prod = __fmul_rn(oma, one_minus_e);
  return __fsub_rn(1.0f, prod);
}

// key(u) + edge: one saturating u32 add and the three-op f32 fold.  The edge
// latency is clamped to LAT32_SAT on upload.
__device__ __forceinline__ uint64_t relax32(uint64_t ku, uint32_t edge_lat, float edge_om) {
  const uint32_t lat = __builtin_elementwise_add_sat(key_lat(ku), edge_lat);
  const float loss = fold_loss(__uint_as_float(key_loss_bits(ku)), edge_om);
  return ((uint64_t)lat << 32) | (uint64_t)__float_as_uint(loss);
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

// Inclusive scans across a wave64 with DPP (row shifts, then the row broadcasts
// of lanes 15 and 31): sum and max of u32.
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
  v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false));
  return v;
}

}  // namespace sg
