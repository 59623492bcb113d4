// gf256.hpp -- host-side GF(2^8) field and matrix algebra for the RS engine.
//
// Product code (no dependency on oracle/).  Field and matrix construction follow
// the codec the reference wraps, github.com/klauspost/reedsolomon v1.12.1
// (go.mod:16): reduction polynomial 0x11d, generator 2 [upstream galois.go];
// encode matrix = vandermonde(K+M, K) x inverse(top K x K) [upstream matrix.go
// buildMatrix]; called from internal/ec/ec.go:26 with K=4, M=2
// (internal/config/config.go:20-23).
//
// Everything here is O(K^2..K^3) per erasure pattern and runs once per pattern
// (cached by the engine); the byte streams never touch this code.
#pragma once

#include <array>
#include <cstdint>
#include <vector>

namespace rs {

struct Field {
  std::array<uint8_t, 512> exp{};
  std::array<uint8_t, 256> log{};
  Field() {
    unsigned x = 1;
    for (int i = 0; i < 255; ++i) {
      exp[i] = static_cast<uint8_t>(x);
      log[x] = static_cast<uint8_t>(i);
      x = (x << 1) ^ ((x & 0x80) ? 0x11d : 0);
      x &= 0xff;
    }
    for (int i = 255; i < 512; ++i) exp[i] = exp[i - 255];
  }
  uint8_t mul(uint8_t a, uint8_t b) const {
    return (a && b) ? exp[log[a] + log[b]] : 0;
  }
  uint8_t inv(uint8_t a) const { return a ? exp[(255 - log[a]) % 255] : 0; }
  // galExp semantics: pow(., 0) = 1, pow(0, n>0) = 0.
  uint8_t pow(uint8_t a, int n) const {
    if (n == 0) return 1;
    if (a == 0) return 0;
    return exp[(static_cast<int>(log[a]) * n) % 255];
  }
};

const Field& field();

// Row-major byte matrix.
struct Matrix {
  int rows = 0, cols = 0;
  std::vector<uint8_t> a;
  Matrix() = default;
  Matrix(int r, int c) : rows(r), cols(c), a(static_cast<size_t>(r) * c, 0) {}
  uint8_t& at(int r, int c) { return a[static_cast<size_t>(r) * cols + c]; }
  uint8_t at(int r, int c) const { return a[static_cast<size_t>(r) * cols + c]; }
};

Matrix multiply(const Matrix& x, const Matrix& y);
// Returns false if singular.
bool invert(const Matrix& in, Matrix* out);
// (K+M) x K systematic encode matrix.
Matrix build_encode_matrix(int k, int m);

}  // namespace rs
