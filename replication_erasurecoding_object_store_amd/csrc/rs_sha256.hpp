// rs_sha256.hpp -- batched SHA-256 launch (rs_sha256.hip), internal to librsgpu.so.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rs {

// Message i: base + offsets[i] (or base + i*stride when offsets is null), lens[i]
// bytes (or len when lens is null).  offsets / lens are device arrays.  Digest i
// (32 bytes, big-endian as FIPS 180-4 prints it) goes to out + 32*i.
// chunk != 0: the message is stored in chunks of `chunk` bytes every `chunk_pitch`
// bytes (a Split object's data shards in a batch slot: byte o of the value lives in
// shard o / S at offset o % S).  lens[i] == ~0: message i is skipped (no digest).
struct Sha256Args {
  const uint8_t* base;
  uint64_t stride;
  const uint64_t* offsets;
  const uint64_t* lens;
  uint64_t len;
  uint32_t n;
  uint8_t* out;
  uint64_t chunk = 0;
  uint64_t chunk_pitch = 0;
};
constexpr uint64_t kSha256Skip = ~0ull;

int launch_sha256(const Sha256Args& a, hipStream_t s);

}  // namespace rs
