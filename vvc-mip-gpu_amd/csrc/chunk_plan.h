// chunk_plan.h -- frames per chunk of one host-API call (mipgpu.cpp search_frames_chunks;
// no HIP dependency, unit-tested by tests/cpp/test_chunk_plan.cpp).
#pragma once
#include <algorithm>
#include <vector>

namespace mipgpu {

// Largest chunk of a call before the transfer caps (mipgpu.cpp search_frames_chunks): a
// slot's frames (`slot_cap`), or -- for a call into an idle pipeline on a small engine
// (three slots) -- half the call, so that its own upload, search and download overlap, but
// never more than a slot holds (a larger chunk would spill into the next slot's region).
inline int call_chunk_cap(int nframes, int slot_cap, int nslots, bool idle) {
  if (nslots == 3 && nframes >= 2 && idle) return std::min(slot_cap, (nframes + 1) / 2);
  return slot_cap;
}

// nframes frames in chunks of at most sb.  `head`: the first chunks ramp up from 4 frames by
// x1.75 (4, 7, 12, 21, ...) while more than sb frames stay for the rest; `tail`: the last
// chunks ramp down the same way (..., 12, 7, 4), again leaving more than sb frames between;
// the rest is cut into equal chunks (sizes differ by at most one frame).  *nhead / *ntail
// (optional): the number of ramp chunks at either end.
inline std::vector<int> chunk_plan(int nframes, int sb, bool head, bool tail, int *nhead = nullptr,
                                   int *ntail = nullptr) {
  std::vector<int> plan, down;
  int left = nframes;
  auto ramp = [&](std::vector<int> &v) {
    for (int c = 4; c < sb && left > sb + c; c = c * 7 / 4) {
      v.push_back(c);
      left -= c;
    }
  };
  if (head) ramp(plan);
  if (nhead) *nhead = (int)plan.size();
  if (tail && left > sb) ramp(down);
  const int nch = (left + sb - 1) / sb;  // the fewest chunks of at most sb, sizes within one
  for (int i = 0; i < nch; i++) plan.push_back(left / nch + (i < left % nch ? 1 : 0));
  if (ntail) *ntail = (int)down.size();
  plan.insert(plan.end(), down.rbegin(), down.rend());
  return plan;
}

}  // namespace mipgpu
