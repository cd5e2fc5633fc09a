// CPU unit test of the host pipeline's chunk plan (csrc/chunk_plan.h): for every call length
// and chunk cap, the chunks cover the call exactly, none exceeds the cap, the unramped part is
// the fewest chunks of at most the cap with sizes within one frame, the ramps are 4, 7, 12, ...
// (reversed at the end), taken only when asked for and only while more than one cap of frames
// stays between them.  Built and run by tests/test_chunk_plan.py (g++, no GPU).
#include <algorithm>
#include <cstdio>
#include <vector>

#include "chunk_plan.h"

static int fails = 0;
#define CHECK(c, ...)                                 \
  do {                                                \
    if (!(c)) {                                       \
      if (fails++ < 20) {                             \
        std::printf("FAIL %s: ", #c);                 \
        std::printf(__VA_ARGS__);                     \
        std::printf("\n");                            \
      }                                               \
    }                                                 \
  } while (0)

int main() {
  const int ramp[] = {4, 7, 12, 21, 36, 63, 110, 192};
  for (int sb = 1; sb <= 96; sb++)
    for (int n = 1; n <= 600; n++)
      for (int mode = 0; mode < 4; mode++) {
        const bool head = mode & 1, tail = mode & 2;
        int h = -1, t = -1;
        const std::vector<int> p = mipgpu::chunk_plan(n, sb, head, tail, &h, &t);
        CHECK(h >= 0 && t >= 0 && h + t <= (int)p.size(), "n %d sb %d mode %d h %d t %d", n, sb, mode, h, t);
        if (fails) break;
        CHECK(head || h == 0, "n %d sb %d: head ramp not asked for", n, sb);
        CHECK(tail || t == 0, "n %d sb %d: tail ramp not asked for", n, sb);
        int sum = 0;
        for (int c : p) {
          CHECK(c >= 1 && c <= sb, "n %d sb %d mode %d chunk %d", n, sb, mode, c);
          sum += c;
        }
        CHECK(sum == n, "n %d sb %d mode %d sum %d", n, sb, mode, sum);
        for (int i = 0; i < h; i++) CHECK(p[i] == ramp[i] && p[i] < sb, "n %d sb %d head[%d] %d", n, sb, i, p[i]);
        for (int i = 0; i < t; i++)
          CHECK(p[p.size() - 1 - i] == ramp[i] && ramp[i] < sb, "n %d sb %d tail[%d] %d", n, sb, i, p[p.size() - 1 - i]);
        int lo = 1 << 30, hi = 0, mid = 0, cnt = 0;
        for (size_t i = h; i + t < p.size(); i++) {
          lo = std::min(lo, p[i]);
          hi = std::max(hi, p[i]);
          mid += p[i];
          cnt++;
        }
        CHECK(cnt >= 1 && hi - lo <= 1, "n %d sb %d mode %d middle %d..%d (%d chunks)", n, sb, mode, lo, hi, cnt);
        CHECK(cnt == (mid + sb - 1) / sb, "n %d sb %d mode %d: %d middle chunks for %d frames", n, sb, mode, cnt, mid);
        CHECK(h + t == 0 || mid > sb, "n %d sb %d mode %d middle %d frames", n, sb, mode, mid);
        // a ramp stops only when its next chunk would not fit or would leave <= sb frames
        if (head && h < 8 && ramp[h] < sb) {
          int after_head = n;
          for (int i = 0; i < h; i++) after_head -= p[i];
          CHECK(!(after_head > sb + ramp[h]), "n %d sb %d: head ramp stopped early at %d", n, sb, h);
        }
      }
  // the call's chunk cap never exceeds a slot (an idle small engine's call of more
  // than two slots' frames had been cut in halves larger than a slot)
  for (int nslots = 3; nslots <= 4; nslots++)
    for (int cap = 1; cap <= 64; cap++)
      for (int n = 1; n <= 300; n++)
        for (int idle = 0; idle < 2; idle++) {
          const int sb = mipgpu::call_chunk_cap(n, cap, nslots, idle);
          CHECK(sb >= 1 && sb <= cap, "n %d cap %d slots %d idle %d: chunk cap %d", n, cap, nslots, idle, sb);
          if (nslots == 3 && idle && n >= 2)
            CHECK(sb == std::min(cap, (n + 1) / 2), "n %d cap %d: idle split %d", n, cap, sb);
          for (int c : mipgpu::chunk_plan(n, sb, false, false)) CHECK(c <= cap, "n %d cap %d: chunk %d", n, cap, c);
        }
  CHECK(mipgpu::call_chunk_cap(3, 1, 3, true) == 1, "max_batch 1, 3 frames");
  CHECK(mipgpu::call_chunk_cap(9, 4, 3, true) == 4, "max_batch 4, 9 frames");
  CHECK(mipgpu::call_chunk_cap(6, 4, 3, true) == 3, "max_batch 4, 6 frames");
  // the shapes documented in DESIGN.md section 6
  CHECK((mipgpu::chunk_plan(128, 64, true, false) == std::vector<int>{4, 7, 12, 21, 42, 42}), "128/64 head");
  CHECK((mipgpu::chunk_plan(128, 64, true, true) == std::vector<int>{4, 7, 12, 21, 37, 36, 7, 4}), "128/64 both");
  CHECK((mipgpu::chunk_plan(64, 16, true, true) == std::vector<int>{4, 7, 12, 9, 9, 12, 7, 4}), "64/16 both");
  CHECK((mipgpu::chunk_plan(16, 3, false, false) == std::vector<int>{3, 3, 3, 3, 2, 2}), "16/3 even");
  if (fails) return 1;
  std::printf("chunk_plan: ok\n");
  return 0;
}
