// Host-side fuzz driver for the product DER parser (minbft_amd/csrc/der.cpp,
// Go encoding/asn1 restatement), built with AddressSanitizer and
// UndefinedBehaviorSanitizer by tests/test_sanitizers.py.  The parser is
// the one host routine that walks untrusted signature bytes; this checks it
// for out-of-bounds reads and undefined behaviour over random and mutated
// encodings (differential parity with the oracle is tests/test_abi.py).
//   der_fuzz ITERATIONS SEED
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "../../include/minbft_gpu.h"

namespace {

std::vector<uint8_t> der_int(std::mt19937_64& g, int len) {
  std::vector<uint8_t> v(len);
  for (auto& b : v) b = (uint8_t)g();
  if (len && (g() & 1)) v[0] &= 0x7f;
  std::vector<uint8_t> out{0x02};
  if (len < 128) {
    out.push_back((uint8_t)len);
  } else {
    out.push_back(0x81);
    out.push_back((uint8_t)len);
  }
  out.insert(out.end(), v.begin(), v.end());
  return out;
}

std::vector<uint8_t> seed_sig(std::mt19937_64& g) {
  auto r = der_int(g, (int)(g() % 40));
  auto s = der_int(g, (int)(g() % 40));
  std::vector<uint8_t> body = r;
  body.insert(body.end(), s.begin(), s.end());
  if (g() % 4 == 0)
    for (int k = (int)(g() % 8); k > 0; k--) body.push_back((uint8_t)g());
  std::vector<uint8_t> out{0x30};
  const size_t n = body.size();
  switch (g() % 4) {
    case 0: out.push_back(0x81); out.push_back((uint8_t)n); break;
    case 1: out.push_back(0x82); out.push_back((uint8_t)(n >> 8)); out.push_back((uint8_t)n); break;
    default: out.push_back((uint8_t)(n & 0xff)); break;
  }
  out.insert(out.end(), body.begin(), body.end());
  if (g() % 3 == 0)
    for (int k = (int)(g() % 6); k > 0; k--) out.push_back((uint8_t)g());
  return out;
}

void mutate(std::mt19937_64& g, std::vector<uint8_t>& v) {
  const int rounds = (int)(g() % 4);
  for (int k = 0; k < rounds && !v.empty(); k++) {
    const size_t at = g() % v.size();
    switch (g() % 5) {
      case 0: v[at] ^= (uint8_t)(1u << (g() % 8)); break;
      case 1: v[at] = (uint8_t)g(); break;
      case 2: v.resize(at); break;
      case 3: v.insert(v.begin() + at, (uint8_t)g()); break;
      default: v[at] = (uint8_t)(0x80 | (g() % 0x8f)); break;  // long-form length bytes
    }
  }
}

}  // namespace

int main(int argc, char** argv) {
  const long iters = argc > 1 ? atol(argv[1]) : 200000;
  std::mt19937_64 g(argc > 2 ? strtoull(argv[2], nullptr, 10) : 1);
  long ok = 0;
  for (long i = 0; i < iters; i++) {
    std::vector<uint8_t> sig;
    if (i % 5 == 0) {
      sig.resize(g() % 96);
      for (auto& b : sig) b = (uint8_t)g();
    } else {
      sig = seed_sig(g);
      mutate(g, sig);
    }
    // exact-size heap copy so that any read past the end is caught
    uint8_t* buf = sig.empty() ? nullptr : (uint8_t*)malloc(sig.size());
    if (buf) memcpy(buf, sig.data(), sig.size());
    uint8_t r[32], s[32];
    size_t consumed = 0;
    const int rc = mbft_der_parse_sig(buf, sig.size(), r, s, &consumed);
    if (rc) {
      ok++;
      if (consumed > sig.size()) {
        fprintf(stderr, "consumed %zu > len %zu at iteration %ld\n", consumed, sig.size(), i);
        return 1;
      }
    }
    free(buf);
  }
  printf("iterations %ld parsed %ld\n", iters, ok);
  return 0;
}
