// ec_service.hpp -- C++ mirror of the reference's internal/ec package over the
// C-ABI in include/rsgpu.h (header-only; link librsgpu.so).
//
// Reference surface, name for name (Go has no toolchain in this image, so the host
// layer above the C-ABI is C++; INTEGRATION.md has the cgo shim for Go):
//   internal/ec/ec.go:15-17   type Service struct { driver reedsolomon.Encoder }
//   internal/ec/ec.go:21-44   func NewService() interfaces.IEcDriver
//   internal/ec/ec.go:48-50   Split(data []byte) ([][]byte, error)
//   internal/ec/ec.go:54-56   Encode(shards [][]byte) error
//   internal/ec/ec.go:59-61   Reconstruct(shards [][]byte) error
//   internal/interfaces/interfaces.go:41-52  IEcDriver
// Go's [][]byte is Shards (a vector of byte vectors, empty == nil); Go's error is
// Error (0 == nil) whose message is klauspost's sentinel text (rs_strerror).
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rsgpu.h"

namespace ec {

constexpr int K = 4;  // internal/config/config.go:21
constexpr int M = 2;  // internal/config/config.go:22

using Shard = std::vector<uint8_t>;
using Shards = std::vector<Shard>;

// A Go []byte: len bytes at p with capacity cap, possibly aliasing a caller's
// buffer (what klauspost's Split hands back); `owner` keeps storage the codec had
// to allocate alive.  len == 0 is Go's nil / empty shard.
struct Slice {
  uint8_t* p = nullptr;
  size_t len = 0, cap = 0;
  std::shared_ptr<std::vector<uint8_t>> owner;
  uint8_t* data() const { return p; }
  size_t size() const { return len; }
  bool empty() const { return len == 0; }
};
using Slices = std::vector<Slice>;

// Go-style error value: code 0 is nil.
struct Error {
  int code = RS_OK;
  explicit operator bool() const { return code != RS_OK; }
  std::string Message() const { return rs_strerror(code); }
  const char* c_str() const { return rs_strerror(code); }
};

// interfaces.IEcDriver (interfaces.go:41-52)
class IEcDriver {
 public:
  virtual ~IEcDriver() = default;
  virtual Error Split(const uint8_t* data, size_t len, Shards* out) = 0;
  virtual Error Encode(Shards& shards) = 0;
  virtual Error Reconstruct(Shards& shards) = 0;
};

class Service final : public IEcDriver {
 public:
  // ec.go:21 NewService(): RS(K, M) on the MI355X engine; device < 0 = one context
  // over every visible GPU (rs_create_multi).  Unlike the reference (which can only
  // fail on bad K/M and then log.Fatalf, ec.go:27-29), this can also report a
  // missing GPU; the caller decides (the Go shim falls back to
  // klauspost).
  static std::unique_ptr<Service> NewService(int k = K, int m = M, int device = 0, Error* err = nullptr) {
    rs_ctx* ctx = nullptr;
    const int rc = device < 0 ? rs_create_multi(k, m, 0, 0, &ctx) : rs_create(k, m, device, 0, &ctx);
    if (err) err->code = rc;
    if (rc != RS_OK) return nullptr;
    std::fprintf(stderr, "[EC Driver] Reed-Solomon k=%d m=%d on %s\n", k, m, rs_backend(ctx));
    return std::unique_ptr<Service>(new Service(ctx, k, m));
  }
  // The same driver with concurrent per-object calls merged into device batches
  // (rs_coalescer_*).  Callers see no difference.
  static std::unique_ptr<Service> NewCoalescingService(int k = K, int m = M, int device = 0,
                                                       const rs_coalescer_opts* opts = nullptr,
                                                       Error* err = nullptr) {
    std::unique_ptr<Service> s = NewService(k, m, device, err);
    if (!s) return s;
    const int rc = rs_coalescer_create(s->ctx_, opts, &s->co_);
    if (err) err->code = rc;
    if (rc != RS_OK) return nullptr;
    return s;
  }
  ~Service() override {
    if (co_) rs_coalescer_destroy(co_);
    rs_destroy(ctx_);
  }
  rs_coalescer* coalescer() const { return co_; }
  Service(const Service&) = delete;
  Service& operator=(const Service&) = delete;

  int DataShards() const { return k_; }
  int ParityShards() const { return m_; }
  rs_ctx* ctx() const { return ctx_; }

  // [upstream reedsolomon.go Split]: perShard = ceil(len/K); data shards carry the
  // payload zero-padded to K*perShard, parity shards are zeroed.  (Go aliases the
  // caller's buffer; the bytes are identical.)
  Error Split(const uint8_t* data, size_t len, Shards* out) override {
    if (len == 0) return Error{RS_ERR_SHORT_DATA};
    const size_t S = rs_shard_size(ctx_, len);
    out->assign(static_cast<size_t>(k_ + m_), Shard(S, 0));
    for (int i = 0; i < k_; ++i) {
      const size_t off = static_cast<size_t>(i) * S;
      if (off < len) {
        const size_t n = len - off < S ? len - off : S;
        std::copy(data + off, data + off + n, (*out)[i].begin());
      }
    }
    return Error{};
  }

  // [upstream reedsolomon.go Split] with Go's aliasing, on a byte vector whose
  // size() is len(data) and capacity() is cap(data): spare capacity is used first
  // (data is resized -- never reallocated -- to min(capacity, (K+M)*perShard) and
  // zero-filled past its old size), so with enough capacity every shard, parity
  // included, is a view into `data`; only shards that do not fit get fresh zeroed
  // storage, the first of them holding the payload's tail.  `data` must outlive
  // the slices and not be reallocated while they are in use.
  Error Split(std::vector<uint8_t>& data, Slices* out) {
    if (data.empty()) return Error{RS_ERR_SHORT_DATA};
    const size_t total = static_cast<size_t>(k_ + m_);
    const size_t data_len = data.size();
    const size_t per = rs_shard_size(ctx_, data_len);
    const size_t need = total * per;
    if (data.capacity() > data.size()) data.resize(std::min(data.capacity(), need), 0);  // within capacity
    out->assign(total, Slice{});
    size_t i = 0;
    for (; i < total && (i + 1) * per <= data.size(); ++i) out->at(i) = Slice{data.data() + i * per, per, per, nullptr};
    if (i < total) {
      auto pad = std::make_shared<std::vector<uint8_t>>((total - i) * per, 0);
      if (data_len > i * per)  // the payload's tail did not fill a whole shard
        std::copy(data.begin() + static_cast<std::ptrdiff_t>(i * per),
                  data.begin() + static_cast<std::ptrdiff_t>(data_len), pad->begin());
      for (size_t j = 0; i + j < total; ++j) out->at(i + j) = Slice{pad->data() + j * per, per, per, pad};
    }
    return Error{};
  }

  // The same on a Go-style slice (e.g. a request body read into an Arena
  // allocation): bytes [len, min(cap, (K+M)*perShard)) are zeroed and used for the
  // shards that fit, exactly as Split(vector&) uses a vector's capacity.
  Error Split(const Slice& data, Slices* out) {
    if (data.empty()) return Error{RS_ERR_SHORT_DATA};
    const size_t total = static_cast<size_t>(k_ + m_);
    const size_t per = rs_shard_size(ctx_, data.len);
    const size_t used = std::max(data.len, std::min(data.cap, total * per));
    std::memset(data.p + data.len, 0, used - data.len);
    out->assign(total, Slice{});
    size_t i = 0;
    for (; i < total && (i + 1) * per <= used; ++i) out->at(i) = Slice{data.p + i * per, per, per, data.owner};
    if (i < total) {
      auto pad = std::make_shared<std::vector<uint8_t>>((total - i) * per, 0);
      if (data.len > i * per) std::copy(data.p + i * per, data.p + data.len, pad->begin());
      for (size_t j = 0; i + j < total; ++j) out->at(i + j) = Slice{pad->data() + j * per, per, per, pad};
    }
    return Error{};
  }

  // Encode / Reconstruct on Go-style slices (the shards Split(vector&) returns).
  Error Encode(Slices& shards) {
    if (static_cast<int>(shards.size()) != k_ + m_) return Error{RS_ERR_TOO_FEW_SHARDS};
    std::vector<uint8_t*> p(shards.size());
    std::vector<size_t> n(shards.size());
    for (size_t i = 0; i < shards.size(); ++i) {
      p[i] = shards[i].p;
      n[i] = shards[i].len;
    }
    return Error{co_ ? rs_co_encode(co_, p.data(), n.data()) : rs_encode(ctx_, p.data(), n.data())};
  }
  // Fills every empty entry (a slice with cap >= the shard size is reused, as
  // klauspost reuses capacity; others get fresh storage).
  Error Reconstruct(Slices& shards) {
    if (static_cast<int>(shards.size()) != k_ + m_) return Error{RS_ERR_TOO_FEW_SHARDS};
    size_t S = 0;
    for (const Slice& s : shards)
      if (!s.empty()) {
        S = s.len;
        break;
      }
    std::vector<uint8_t*> p(shards.size());
    std::vector<size_t> n(shards.size());
    for (size_t i = 0; i < shards.size(); ++i) {
      Slice& s = shards[i];
      if (s.empty() && S > 0 && s.cap < S) {
        s.owner = std::make_shared<std::vector<uint8_t>>(S, 0);
        s.p = s.owner->data();
        s.cap = S;
      }
      p[i] = s.p;
      n[i] = s.len;
    }
    Error e{co_ ? rs_co_reconstruct(co_, p.data(), n.data()) : rs_reconstruct(ctx_, p.data(), n.data())};
    if (e) return e;
    for (size_t i = 0; i < shards.size(); ++i)
      if (shards[i].empty() && n[i] == S) shards[i].len = S;
    return e;
  }

  Error Encode(Shards& shards) override {
    if (static_cast<int>(shards.size()) != k_ + m_) return Error{RS_ERR_TOO_FEW_SHARDS};
    std::vector<uint8_t*> p(shards.size());
    std::vector<size_t> n(shards.size());
    for (size_t i = 0; i < shards.size(); ++i) {
      p[i] = shards[i].empty() ? nullptr : shards[i].data();
      n[i] = shards[i].size();
    }
    return Error{co_ ? rs_co_encode(co_, p.data(), n.data()) : rs_encode(ctx_, p.data(), n.data())};
  }

  // Fills every empty (nil) entry, data and parity (readservice.go:285 and
  // poller.go:282 rely on it).
  Error Reconstruct(Shards& shards) override { return reconstruct(shards, false); }
  Error ReconstructData(Shards& shards) { return reconstruct(shards, true); }

  // Encode plus the write path's cold_hash (writeservice.go:222 and :267,
  // computeSHA256Hex(value) :51-54) in one coalesced GPU batch: digest = SHA-256 of
  // the first value_len bytes of data shards 0..K-1 (the Split input); needs the
  // coalescing service (RS_ERR_NOT_SUPPORTED without).  The GPU digest is one lane
  // per object (rs_co_encode_hash): it pays for bulk loads of many small values, not
  // per request -- the Go shim's EncodeHash hashes on the CPU while the GPU encodes
  // (rsgpu.h).
  Error EncodeHash(Shards& shards, size_t value_len, uint8_t digest[32]) {
    if (!co_) return Error{RS_ERR_NOT_SUPPORTED};
    if (static_cast<int>(shards.size()) != k_ + m_) return Error{RS_ERR_TOO_FEW_SHARDS};
    std::vector<uint8_t*> p(shards.size());
    std::vector<size_t> n(shards.size());
    for (size_t i = 0; i < shards.size(); ++i) {
      p[i] = shards[i].empty() ? nullptr : shards[i].data();
      n[i] = shards[i].size();
    }
    return Error{rs_co_encode_hash(co_, p.data(), n.data(), value_len, digest)};
  }

  // The same on Go-style slices: Split(const Slice&) of an Arena body gives
  // contiguous data shards, so the batch hashes the value where it lies (in place).
  Error EncodeHash(Slices& shards, size_t value_len, uint8_t digest[32]) {
    if (!co_) return Error{RS_ERR_NOT_SUPPORTED};
    if (static_cast<int>(shards.size()) != k_ + m_) return Error{RS_ERR_TOO_FEW_SHARDS};
    std::vector<uint8_t*> p(shards.size());
    std::vector<size_t> n(shards.size());
    for (size_t i = 0; i < shards.size(); ++i) {
      p[i] = shards[i].p;
      n[i] = shards[i].len;
    }
    return Error{rs_co_encode_hash(co_, p.data(), n.data(), value_len, digest)};
  }

  // [upstream Verify]
  Error Verify(const Shards& shards, bool* ok) {
    if (static_cast<int>(shards.size()) != k_ + m_) return Error{RS_ERR_TOO_FEW_SHARDS};
    std::vector<uint8_t*> p(shards.size());
    std::vector<size_t> n(shards.size());
    for (size_t i = 0; i < shards.size(); ++i) {
      p[i] = const_cast<uint8_t*>(shards[i].data());
      n[i] = shards[i].size();
    }
    int v = 0;
    Error e{co_ ? rs_co_verify(co_, p.data(), n.data(), &v) : rs_verify(ctx_, p.data(), n.data(), &v)};
    *ok = v != 0;
    return e;
  }

 private:
  Service(rs_ctx* c, int k, int m) : ctx_(c), k_(k), m_(m) {}

  Error reconstruct(Shards& shards, bool data_only) {
    if (static_cast<int>(shards.size()) != k_ + m_) return Error{RS_ERR_TOO_FEW_SHARDS};
    size_t S = 0;
    for (const Shard& s : shards)
      if (!s.empty()) {
        S = s.size();
        break;
      }
    std::vector<uint8_t*> p(shards.size());
    std::vector<size_t> n(shards.size());
    std::vector<Shard> fresh(shards.size());
    for (size_t i = 0; i < shards.size(); ++i) {
      if (shards[i].empty()) {
        fresh[i].assign(S ? S : 1, 0);  // Go: make([]byte, shardSize)
        p[i] = fresh[i].data();
        n[i] = 0;
      } else {
        p[i] = shards[i].data();
        n[i] = shards[i].size();
      }
    }
    int rc;
    if (co_)
      rc = data_only ? rs_co_reconstruct_data(co_, p.data(), n.data()) : rs_co_reconstruct(co_, p.data(), n.data());
    else
      rc = data_only ? rs_reconstruct_data(ctx_, p.data(), n.data()) : rs_reconstruct(ctx_, p.data(), n.data());
    Error e{rc};
    if (e) return e;
    for (size_t i = 0; i < shards.size(); ++i)
      if (shards[i].empty() && n[i] == S && S > 0) {
        fresh[i].resize(S);
        shards[i] = std::move(fresh[i]);
      }
    return e;
  }

  rs_ctx* ctx_;
  rs_coalescer* co_ = nullptr;
  int k_, m_;
};

// The Go shim's Arena (ec_gpu.go): slices backed by page-locked memory the
// context owns (rs_host_alloc: pinned by the driver for life, the only host memory
// the kernels address in place), so a coalesced call whose shards -- read and
// filled -- all come from an arena runs in place on the GPU: no staging copy of the
// request body, parity written straight into the caller's slices.  Allocations are
// 16-B aligned (the in-place kernel's condition); anything else is staged as usual.
class Arena {
 public:
  static std::unique_ptr<Arena> New(const Service& svc, size_t size, Error* err = nullptr) {
    const size_t n = (size + 4095) & ~size_t(4095);
    void* p = nullptr;
    const int rc = n ? rs_host_alloc(svc.ctx(), n, &p) : RS_ERR_INVALID_ARG;
    if (err) err->code = rc;
    if (rc != RS_OK) return nullptr;
    return std::unique_ptr<Arena>(new Arena(svc.ctx(), static_cast<uint8_t*>(p), n));
  }
  ~Arena() { rs_host_free(ctx_, base_); }
  Arena(const Arena&) = delete;
  Arena& operator=(const Arena&) = delete;

  // n bytes (len = cap = n), 16-B aligned; an empty slice when the arena is full.
  Slice Alloc(size_t n) {
    std::lock_guard<std::mutex> g(mu_);
    if (n == 0 || n > size_ - off_) return Slice{};
    Slice s{base_ + off_, n, n, nullptr};
    off_ = std::min(size_, off_ + ((n + 15) & ~size_t(15)));
    return s;
  }
  // Every earlier Alloc is invalid afterwards.
  void Reset() {
    std::lock_guard<std::mutex> g(mu_);
    off_ = 0;
  }
  size_t Size() const { return size_; }

 private:
  Arena(rs_ctx* c, uint8_t* b, size_t n) : ctx_(c), base_(b), size_(n) {}
  rs_ctx* ctx_;
  uint8_t* base_;
  size_t size_, off_ = 0;
  std::mutex mu_;
};

}  // namespace ec
