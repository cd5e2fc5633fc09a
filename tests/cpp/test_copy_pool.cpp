// Unit test of the bounce ring's parallel memcpy (vvc-mip-gpu_amd/csrc/copy_pool.h), no GPU:
// every byte of copies of many sizes lands, back-to-back jobs do not mix (a worker that wakes
// late claims nothing of a later job), and the caller finishes a copy alone when every pool
// thread is busy elsewhere (here: all threads held up before the job starts).
#include "copy_pool.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

static int fails = 0;
#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);     \
      fails++;                                                    \
    }                                                             \
  } while (0)

int main() {
  using mipgpu::CopyPool;
  std::vector<unsigned char> src(40u << 20), dst(40u << 20);
  for (size_t i = 0; i < src.size(); i++) src[i] = (unsigned char)(i * 2654435761u >> 13);
  {
    CopyPool pool(8);
    // sizes around the chunk and parallel thresholds, odd tails
    const size_t sizes[] = {1, 4095, CopyPool::kMinParallel - 1, CopyPool::kMinParallel,
                            CopyPool::kMinParallel + 1, 5 * CopyPool::kChunk + 17, 39u << 20};
    for (int rep = 0; rep < 20; rep++)
      for (size_t n : sizes) {
        const size_t off = (rep * 4099) % 8192;
        std::fill(dst.begin(), dst.end(), 0xA5);
        pool.copy(dst.data() + off, src.data(), n);
        CHECK(std::memcmp(dst.data() + off, src.data(), n) == 0);
        CHECK(off == 0 || dst[off - 1] == 0xA5);
        CHECK(off + n >= dst.size() || dst[off + n] == 0xA5);
      }
    // many small jobs back to back (workers wake up late relative to the jobs)
    for (int rep = 0; rep < 2000; rep++) {
      const size_t n = CopyPool::kMinParallel + (rep % 7) * 12345;
      pool.copy(dst.data(), src.data() + rep, n);
      if (rep % 97 == 0) CHECK(std::memcmp(dst.data(), src.data() + rep, n) == 0);
    }
    CHECK(std::memcmp(dst.data(), src.data() + 1999, CopyPool::kMinParallel + (1999 % 7) * 12345) == 0);
  }
  {
    // no pool threads at all: the caller copies everything
    CopyPool pool(0);
    pool.copy(dst.data(), src.data(), 39u << 20);
    CHECK(std::memcmp(dst.data(), src.data(), 39u << 20) == 0);
  }
  if (fails) return 1;
  std::printf("copy_pool: ok\n");
  return 0;
}
