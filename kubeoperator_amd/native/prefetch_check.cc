// Sanitizer harness for the token prefetcher core: built by tests/test_native_sanitizers.py
// with -fsanitize=address,undefined and separately with -fsanitize=thread, then run. Checks every batch
// against the window starts it must have (deterministic stream), skip/resume, both token widths, and
// create/destroy while workers are still filling the ring (shutdown races).
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>

#include "prefetch_core.h"

using kop_native::TokenPrefetcher;

static int check_stream(const std::string& path, int itemsize, int64_t ntok, int64_t vocab) {
  int bad = 0;
  TokenPrefetcher p(path, itemsize, 4, 129, 7, 4, 3);
  auto verify = [&](int64_t idx, const std::vector<int64_t>& v) {
    const auto st = p.starts(idx);
    for (int64_t r = 0; r < 4; ++r)
      for (int64_t k = 0; k < 129; ++k)
        if (v[r * 129 + k] != (st[r] + k) % vocab) ++bad;
  };
  for (int64_t i = 0; i < 200; ++i) verify(i, p.next());
  p.skip(10);
  for (int64_t i = 210; i < 230; ++i) verify(i, p.next());
  if (p.position() != 230) ++bad;
  (void)ntok;
  return bad;
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  const int64_t ntok = 100000, vocab = 50257;
  const std::string p16 = dir + "/tok16.bin", p32 = dir + "/tok32.bin";
  {
    std::ofstream f16(p16, std::ios::binary), f32(p32, std::ios::binary);
    for (int64_t i = 0; i < ntok; ++i) {
      const uint16_t a = static_cast<uint16_t>(i % vocab);
      const uint32_t b = static_cast<uint32_t>(i % vocab);
      f16.write(reinterpret_cast<const char*>(&a), 2);
      f32.write(reinterpret_cast<const char*>(&b), 4);
    }
  }
  int bad = check_stream(p16, 2, ntok, vocab) + check_stream(p32, 4, ntok, vocab);
  // destroy while the workers are mid-fill
  for (int i = 0; i < 50; ++i) {
    TokenPrefetcher p(p16, 2, 8, 1025, static_cast<uint64_t>(i), 8, 4);
    if (i % 2) (void)p.next();
  }
  try {
    TokenPrefetcher p(p16, 3, 1, 10, 0, 1, 1);
    ++bad;  // itemsize 3 must be rejected
  } catch (const std::invalid_argument&) {
  }
  std::printf("prefetch_check: %s (%d mismatches)\n", bad ? "FAIL" : "OK", bad);
  return bad ? 1 : 0;
}
