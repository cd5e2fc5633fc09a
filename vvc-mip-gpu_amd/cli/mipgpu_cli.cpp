// mipgpu_cli.cpp -- command-line front end replacing the reference's main.cpp.
//
// Same flags as main.cpp:51-59 (boost::program_options style, including unambiguous
// long-option prefixes such as --Filter=...):
//   -h/--help  --DeviceIndex N  -f/--FramesToBeEncoded N  -s/--Resolution WxH
//   -o/--OriginalFrames file.csv  -l/--OutputPreffix prefix  --FilterType name  --KernelIdx K
// Same input format (CSV: H lines of W comma-separated samples per frame, frames
// concatenated, main.cpp:364-384), same cost log (<prefix>.csv, header
// "CTU,cuSizeName,W,H,CU,X,Y,Mode,SAD,SATD,minSadHad", one row per (CTU, shape, CU, mode)
// for frame 0, main_aux_functions.h:735-798) and the same timing line
// ("Elapsed time (ms) from writing samples to reading distortion (Nx), T",
// main_aux_functions.h:908-914).  In the reference's default build
// (MAX_PERFORMANCE_DIST=1) the SAD/SATD columns print never-written memory (0 in
// practice); this CLI prints 0 there too unless --ReportSadSatd is given.
// Extensions: --ReportSadSatd, --AllFrames (log every frame, column CTU stays per frame,
// a Frame column is NOT added to keep the format), --BestModes file (per-CU decision),
// --TopK K (the BestModes file lists each CU's K best modes, one row per rank),
// --BinaryLog file (every frame's int32 cost table, mipgpu/layout.py read_binary_log),
// --InputFormat csv|u16|yuv420p10 (raw little-endian 16-bit luma frames, or planar
// 4:2:0 10-bit YUV of which the luma plane is used; auto: by file extension),
// --BatchFrames N, --Threads N (log formatting threads), and --DeviceIndex accepting a
// list ("0,1,2,3"): the frames are sharded over those GPUs, one engine and one host thread
// per device (frames are independent; no inter-GPU communication).
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <memory>
#include <string>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "mipgpu.h"

namespace {

const char *kFilters[] = {"filterFrame_1d_int", "filterFrame_1d_float", "filterFrame_2d_int_quarterCtu",
                          "filterFrame_2d_float_quarterCtu", "filterFrame_1d_int_5x5", "filterFrame_1d_float_5x5",
                          "filterFrame_2d_int_5x5_quarterCtu", "filterFrame_2d_float_5x5_quarterCtu"};

struct Options {
  int frames = -1, kernel_idx = 0, batch = 0, threads = 0, topk = 1;  // batch 0: auto
  std::vector<int> devices{0};
  std::string device_arg = "0";
  bool device_set = false, prefix_set = false, kidx_set = false, help = false;
  bool sad_satd = false, all_frames = false, strict_res = false;
  std::string resolution, input, prefix, filter, best_modes, binary_log, input_format = "auto";
};

struct OptDef {
  const char *name;
  char shortname;
  bool takes_value;
};
const OptDef kOpts[] = {{"help", 'h', false},        {"DeviceIndex", 0, true},   {"FramesToBeEncoded", 'f', true},
                        {"Resolution", 's', true},   {"OriginalFrames", 'o', true}, {"OutputPreffix", 'l', true},
                        {"FilterType", 0, true},     {"KernelIdx", 0, true},     {"ReportSadSatd", 0, false},
                        {"AllFrames", 0, false},     {"BestModes", 0, true},     {"BatchFrames", 0, true},
                        {"Threads", 0, true},        {"TopK", 0, true},          {"BinaryLog", 0, true},
                        {"InputFormat", 0, true},    {"StrictResolution", 0, false}};

void usage() {
  std::cout << "Allowed options:\n"
               "  -h [ --help ]                     produce help message\n"
               "  --DeviceIndex arg (=0)            Index of the GPU device (or a list: frames are sharded)\n"
               "  -f [ --FramesToBeEncoded ] arg    Number of frames to be processed\n"
               "  -s [ --Resolution ] arg           Resolution of the video, in the format 1920x1080\n"
               "  -o [ --OriginalFrames ] arg       Input file for original frames samples\n"
               "  -l [ --OutputPreffix ] arg (=\"\")  Output files preffix with produced costs\n"
               "  --FilterType arg                  Type of smoothing filter\n"
               "  --KernelIdx arg (=0)              Index of the filtering kernel used to define the coefficients\n"
               "  --ReportSadSatd                   Log real SAD/SATD columns (reference: MAX_PERFORMANCE_DIST=0)\n"
               "  --AllFrames                       Log every frame (reference logs frame 0 only)\n"
               "  --BestModes arg                   Write the per-CU best mode / cost to this CSV\n"
               "  --BatchFrames arg (=auto)         Frames per device batch (auto: ~256 MB of samples, at most 32)\n"
               "  --Threads arg (=0)                CSV parsing / log-formatting threads (0 = all cores)\n"
               "  --TopK arg (=1)                   Modes per CU in the BestModes file (1..32, ranked)\n"
               "  --BinaryLog arg                   Write every frame's int32 cost table to this file\n"
               "  --InputFormat arg (=auto)         csv | u16 (raw 16-bit luma) | yuv420p10 (planar 4:2:0, 10 bit)\n"
               "  --StrictResolution                Accept only the reference's resolutions (constants.h:17-23)\n";
}

int set_opt(Options &o, const std::string &name, const std::string &val) {
  try {
    if (name == "help") o.help = true;
    else if (name == "DeviceIndex") {
      o.devices.clear();
      std::stringstream ss(val);
      std::string item;
      while (std::getline(ss, item, ',')) o.devices.push_back(std::stoi(item));
      if (o.devices.empty()) throw std::invalid_argument("empty device list");
      o.device_arg = val;
      o.device_set = true;
    }
    else if (name == "FramesToBeEncoded") o.frames = std::stoi(val);
    else if (name == "Resolution") o.resolution = val;
    else if (name == "OriginalFrames") o.input = val;
    else if (name == "OutputPreffix") o.prefix = val, o.prefix_set = true;
    else if (name == "FilterType") o.filter = val;
    else if (name == "KernelIdx") o.kernel_idx = std::stoi(val), o.kidx_set = true;
    else if (name == "ReportSadSatd") o.sad_satd = true;
    else if (name == "AllFrames") o.all_frames = true;
    else if (name == "StrictResolution") o.strict_res = true;
    else if (name == "BestModes") o.best_modes = val;
    else if (name == "BatchFrames") o.batch = val == "auto" ? 0 : std::max(1, std::stoi(val));
    else if (name == "Threads") o.threads = std::stoi(val);
    else if (name == "TopK") {
      o.topk = std::stoi(val);
      if (o.topk < 1 || o.topk > 32) throw std::invalid_argument("TopK");
    }
    else if (name == "BinaryLog") o.binary_log = val;
    else if (name == "InputFormat") {
      if (val != "auto" && val != "csv" && val != "u16" && val != "yuv420p10") throw std::invalid_argument("format");
      o.input_format = val;
    }
  } catch (...) {
    std::cerr << "the argument ('" << val << "') for option '--" << name << "' is invalid\n";
    return 1;
  }
  return 0;
}

// boost-like parsing: --name=value, --name value, unambiguous prefixes, -x value, -xvalue.
int parse(int argc, char **argv, Options &o) {
  for (int i = 1; i < argc; i++) {
    std::string a = argv[i], name, val;
    bool have_val = false;
    const OptDef *def = nullptr;
    if (a.rfind("--", 0) == 0) {
      std::string body = a.substr(2);
      const size_t eq = body.find('=');
      if (eq != std::string::npos) val = body.substr(eq + 1), body = body.substr(0, eq), have_val = true;
      std::vector<const OptDef *> hits;
      for (const OptDef &d : kOpts) {
        if (body == d.name) { hits = {&d}; break; }
        if (std::string(d.name).rfind(body, 0) == 0) hits.push_back(&d);
      }
      if (hits.size() != 1) {
        std::cerr << (hits.empty() ? "unrecognised option '" : "option '") << a
                  << (hits.empty() ? "'\n" : "' is ambiguous\n");
        return 1;
      }
      def = hits[0];
    } else if (a.size() >= 2 && a[0] == '-') {
      for (const OptDef &d : kOpts)
        if (d.shortname == a[1]) def = &d;
      if (!def) { std::cerr << "unrecognised option '" << a << "'\n"; return 1; }
      if (a.size() > 2) val = a.substr(2), have_val = true;
    } else {
      std::cerr << "unexpected positional argument '" << a << "'\n";
      return 1;
    }
    if (def->takes_value && !have_val) {
      if (i + 1 >= argc) { std::cerr << "the required argument for option '--" << def->name << "' is missing\n"; return 1; }
      val = argv[++i];
    }
    if (set_opt(o, def->name, val)) return 1;
  }
  return 0;
}

// main_aux_functions.h:113-162
int report_parameters(const Options &o, bool alt) {
  int errors = 0;
  std::cout << "-=-= INPUT PARAMETERS =-=-" << std::endl;
  if (!o.device_set) std::cout << "  Device index not set. Using standard value of " << o.device_arg << "." << std::endl;
  else std::cout << "  Device Index=" << o.device_arg << std::endl;
  if (!o.prefix_set) std::cout << "  OutputPreffix log file not set. The output will not be written to any file." << std::endl;
  else std::cout << "  OutputPreffix=" << o.prefix << std::endl;
  if (o.frames >= 0) std::cout << "  FramesToBeEncoded=" << o.frames << std::endl;
  else { std::cout << "  [!] ERROR: FramesToBeEncoded not set." << std::endl; errors++; }
  if (!o.input.empty()) std::cout << "  InputOriginalFrame=" << o.input << std::endl;
  else { std::cout << "  [!] ERROR: Input original frames not set." << std::endl; errors++; }
  if (alt) {
    std::cout << "  FilterType=" << o.filter << std::endl;
    if (!o.kidx_set) std::cout << "  KernelIdx not set. Using default value zero." << std::endl;
    else std::cout << "  KernelIdx=" << o.kernel_idx << std::endl;
  }
  return errors;
}

// Page-locked host buffer (mip_host_alloc): the engine's transfers run at DMA rate.  With one
// device, on that GPU's NUMA node (mip_host_alloc_near).
template <class T>
struct Pinned {
  T *p = nullptr;
  size_t n = 0;
  bool alloc(size_t count, int near_device = -1) {
    void *v = nullptr;
    if ((near_device >= 0 ? mip_host_alloc_near(near_device, count * sizeof(T), &v) : mip_host_alloc(count * sizeof(T), &v)) != 0)
      return false;
    p = static_cast<T *>(v);
    n = count;
    return true;
  }
  ~Pinned() { mip_host_free(p); }
  T *data() { return p; }
  bool empty() const { return n == 0; }
  T &operator[](size_t i) { return p[i]; }
};

// Sequential frame source (main.cpp:364-384 reads the whole CSV before the search; here
// frames are read chunk by chunk while earlier chunks are searched and logged, so host
// memory does not grow with the sequence length).
//  * CSV: the file is memory-mapped; per chunk the H*n line starts are indexed and the rows
//    parsed by `threads` threads (H lines of W comma-separated samples per frame).
//  * raw: `luma_only` = consecutive W x H little-endian 16-bit frames; otherwise planar
//    4:2:0 with 16-bit samples (yuv420p10le), whose two chroma planes (W/2 x H/2 each) are
//    skipped.
// Samples above 10 bits break the engine's input contract (include/mipgpu.h): the row's first
// such column goes to *bad_x (the engine would report the frame too, after its search).
bool parse_row(const char *p, const char *end, int W, uint16_t *out, int *bad_x) {
  for (int x = 0; x < W; x++) {
    while (p < end && (*p == ' ' || *p == '\r')) p++;
    long long v = 0;
    bool any = false;
    while (p < end && *p >= '0' && *p <= '9') v = std::min(v * 10 + (*p++ - '0'), 1LL << 40), any = true;
    if (!any) return false;
    if (v > 1023 && *bad_x < 0) *bad_x = x;
    out[x] = (uint16_t)v;
    while (p < end && *p != ',' && *p != '\n') p++;
    if (p < end && *p == ',') p++;
  }
  return true;
}

class FrameSource {
 public:
  ~FrameSource() {
    if (map_ && map_ != MAP_FAILED) munmap(map_, size_);
    if (fd_ >= 0) close(fd_);
    if (raw_) fclose(raw_);
  }
  bool open(const std::string &path, const std::string &fmt, int W, int H, int threads) {
    W_ = W, H_ = H, threads_ = std::max(1, threads);
    csv_ = fmt == "csv";
    if (!csv_) {
      luma_only_ = fmt == "u16";
      raw_ = fopen(path.c_str(), "rb");
      return raw_ != nullptr;
    }
    fd_ = ::open(path.c_str(), O_RDONLY);
    if (fd_ < 0) return false;
    struct stat st;
    if (fstat(fd_, &st) != 0) return false;
    size_t sz = (size_t)st.st_size;
    if (sz == 0) return true;  // empty file: the first read fails
    map_ = mmap(nullptr, sz, PROT_READ, MAP_PRIVATE, fd_, 0);
    if (map_ == MAP_FAILED) return false;
    size_ = sz;
    madvise(map_, size_, MADV_SEQUENTIAL);
    return true;
  }
  // Next n frames into out (n * W * H samples).
  bool read(int n, uint16_t *out) {
    const size_t fs = (size_t)W_ * H_;
    if (!csv_) {
      const size_t chroma = luma_only_ ? 0 : 2 * (size_t)(W_ / 2) * (H_ / 2);
      for (int i = 0; i < n; i++) {
        if (fread(out + i * fs, 2, fs, raw_) != fs) return false;
        if (chroma && fseek(raw_, (long)(chroma * 2), SEEK_CUR) != 0) return false;
      }
      return true;
    }
    const char *data = static_cast<const char *>(map_);
    const size_t rows = (size_t)H_ * n;
    start_.clear();
    for (size_t r = 0; r < rows; r++) {
      if (pos_ >= size_) return false;
      start_.push_back(pos_);
      const void *nl = memchr(data + pos_, '\n', size_ - pos_);
      pos_ = nl ? (size_t)((const char *)nl - data) + 1 : size_;
    }
    start_.push_back(pos_);
    std::vector<char> ok(threads_, 1);
    std::vector<long long> bad(threads_, -1);  // first out-of-range sample per thread (row * W + x)
    std::vector<std::thread> pool;
    for (int t = 0; t < threads_; t++)
      pool.emplace_back([&, t] {
        for (size_t r = t; r < rows; r += threads_) {
          int bx = -1;
          if (!parse_row(data + start_[r], data + start_[r + 1], W_, out + r * W_, &bx)) ok[t] = 0;
          if (bx >= 0 && bad[t] < 0) bad[t] = (long long)r * W_ + bx;
        }
      });
    for (auto &th : pool) th.join();
    for (long long b : bad)
      if (b >= 0 && (range_bad_ < 0 || b + frames_read_ * (long long)fs < range_bad_))
        range_bad_ = b + frames_read_ * (long long)fs;
    frames_read_ += n;
    if (range_bad_ >= 0) return false;
    return std::all_of(ok.begin(), ok.end(), [](char c) { return c != 0; });
  }
  // First sample above 10 bits (frame * W * H + row * W + x), or -1.
  long long range_error() const { return range_bad_; }

 private:
  int W_ = 0, H_ = 0, threads_ = 1;
  bool csv_ = true, luma_only_ = true;
  FILE *raw_ = nullptr;
  int fd_ = -1;
  void *map_ = nullptr;
  size_t size_ = 0, pos_ = 0;
  std::vector<size_t> start_;
  long long range_bad_ = -1, frames_read_ = 0;
};

std::string input_format(const Options &o) {
  if (o.input_format != "auto") return o.input_format;
  auto ends = [&](const char *suf) {
    const size_t n = strlen(suf);
    return o.input.size() >= n && o.input.compare(o.input.size() - n, n, suf) == 0;
  };
  if (ends(".yuv")) return "yuv420p10";
  if (ends(".u16") || ends(".raw")) return "u16";
  return "csv";
}

inline char *put_int(char *p, long long v) {
  char tmp[24];
  int n = 0;
  const bool neg = v < 0;
  unsigned long long u = neg ? (unsigned long long)(-v) : (unsigned long long)v;
  do tmp[n++] = (char)('0' + u % 10); while (u /= 10);
  if (neg) *p++ = '-';
  while (n) *p++ = tmp[--n];
  return p;
}

struct ShapeInfo {
  int w, h, modes, ncu, off;
  std::string name;
  std::vector<int> x, y;
};

// Rows formatted by CTU chunks on up to kMaxLiveChunks threads, written in chunk order.  Host
// memory is bounded independently of the thread count: at most kMaxLiveChunks chunk buffers
// exist, each allocated once without zero-filling (only the pages a chunk's rows touch are
// committed -- ~55 bytes per row against the chunk_bytes bound), and reused round after
// round (an 8K frame's cost log is ~11 GB of text).
// format(c, p) writes chunk c's rows at p and returns the end; chunk_bytes bounds them.
constexpr int kMaxLiveChunks = 16;
template <class F>
void write_chunks_in_order(FILE *fp, int nchunks, size_t chunk_bytes, int threads, F &&format) {
  const int nt = std::max(1, std::min({threads, kMaxLiveChunks, nchunks}));
  std::vector<std::unique_ptr<char[]>> bufs(nt);
  std::vector<size_t> used(nt);
  for (int c0 = 0; c0 < nchunks; c0 += nt) {
    const int n = std::min(nt, nchunks - c0);
    std::vector<std::thread> pool;
    for (int t = 0; t < n; t++)
      pool.emplace_back([&, t] {
        if (!bufs[t]) bufs[t].reset(new char[chunk_bytes]);  // default-initialised: no zero fill
        used[t] = format(c0 + t, bufs[t].get()) - bufs[t].get();
      });
    for (auto &th : pool) th.join();
    for (int t = 0; t < n; t++) fwrite(bufs[t].get(), 1, used[t], fp);
  }
}

// Bound on a row of either format: every int field at its widest (11 characters; W, H, CU,
// Mode, Rank, Transposed are shorter), a shape name of <= 16 characters, separators and the
// newline: <= 102 bytes for a cost-log row, <= 95 for a decision row.
constexpr size_t kMaxRowBytes = 128;

// exportAllDistortionValues_File (main_aux_functions.h:735-798).
void write_cost_log(FILE *fp, const std::vector<ShapeInfo> &shapes, int nctus, int W, const int32_t *cost,
                    const int32_t *sad, const int32_t *satd, int threads) {
  const int ctu_cols = (W + 127) / 128;
  const int chunk = 2;  // CTUs per chunk: 195 680 rows, <= 25 MB of buffer bound
  const int nchunks = (nctus + chunk - 1) / chunk;
  write_chunks_in_order(fp, nchunks, (size_t)chunk * MIP_COSTS_PER_CTU_ABI * kMaxRowBytes, threads, [&](int c, char *p) {
    for (int ctu = c * chunk; ctu < std::min(nctus, (c + 1) * chunk); ctu++) {
      const int cx = 128 * (ctu % ctu_cols), cy = 128 * (ctu / ctu_cols);
      for (const ShapeInfo &sh : shapes)
        for (int cu = 0; cu < sh.ncu; cu++)
          for (int m = 0; m < 2 * sh.modes; m++) {
            const size_t idx = (size_t)ctu * MIP_COSTS_PER_CTU_ABI + sh.off + (size_t)cu * 2 * sh.modes + m;
            p = put_int(p, ctu); *p++ = ',';
            memcpy(p, sh.name.data(), sh.name.size()); p += sh.name.size(); *p++ = ',';
            p = put_int(p, sh.w); *p++ = ',';
            p = put_int(p, sh.h); *p++ = ',';
            p = put_int(p, cu); *p++ = ',';
            p = put_int(p, cx + sh.x[cu]); *p++ = ',';
            p = put_int(p, cy + sh.y[cu]); *p++ = ',';
            p = put_int(p, m); *p++ = ',';
            p = put_int(p, sad ? sad[idx] : 0); *p++ = ',';
            p = put_int(p, satd ? satd[idx] : 0); *p++ = ',';
            p = put_int(p, cost[idx]); *p++ = '\n';
          }
    }
    return p;
  });
}

// Decision rows of one frame (--BestModes): K = 1 "Frame,CTU,cuSizeName,W,H,CU,X,Y,BestMode,
// Transposed,Cost", K > 1 one row per rank "...,Rank,Mode,Transposed,Cost" (modes past the
// CU's list omitted, unavailable CUs one row with -1), formatted like the cost log.
void write_best_rows(FILE *fp, const std::vector<ShapeInfo> &shapes, int nctus, int ctu_cols, int frame, int K,
                     const uint8_t *best, const int32_t *best_cost, int threads) {
  const int chunk = 8;
  const int nchunks = (nctus + chunk - 1) / chunk;
  write_chunks_in_order(fp, nchunks, (size_t)chunk * MIP_CUS_PER_CTU_ABI * K * kMaxRowBytes, threads, [&](int c, char *p) {
    for (int ctu = c * chunk; ctu < std::min(nctus, (c + 1) * chunk); ctu++) {
      size_t k = (size_t)ctu * MIP_CUS_PER_CTU_ABI;
      for (const ShapeInfo &sh : shapes)
        for (int cu = 0; cu < sh.ncu; cu++, k++) {
          const size_t i0 = k * K;
          const int x = 128 * (ctu % ctu_cols) + sh.x[cu], y = 128 * (ctu / ctu_cols) + sh.y[cu];
          for (int r = 0; r < K; r++) {
            const int m = best[i0 + r];
            if (K > 1 && m == 0xff && best[i0] != 0xff) break;  // past the CU's modes
            p = put_int(p, frame); *p++ = ',';
            p = put_int(p, ctu); *p++ = ',';
            memcpy(p, sh.name.data(), sh.name.size()); p += sh.name.size(); *p++ = ',';
            p = put_int(p, sh.w); *p++ = ',';
            p = put_int(p, sh.h); *p++ = ',';
            p = put_int(p, cu); *p++ = ',';
            p = put_int(p, x); *p++ = ',';
            p = put_int(p, y); *p++ = ',';
            if (K > 1) { p = put_int(p, r); *p++ = ','; }
            p = put_int(p, m == 0xff ? -1 : m % sh.modes); *p++ = ',';
            p = put_int(p, m == 0xff ? -1 : (m >= sh.modes)); *p++ = ',';
            p = put_int(p, best_cost[i0 + r]); *p++ = '\n';
            if (m == 0xff) break;  // unavailable CU: one row
          }
        }
    }
    return p;
  });
}

}  // namespace

int main(int argc, char **argv) {
  Options o;
  if (parse(argc, argv, o)) return 1;
  if (o.help) { usage(); return 1; }  // main.cpp:64-67 returns 1 after help
  const bool alt = !o.filter.empty();
  const int errors = report_parameters(o, alt);
  int filter = MIP_FILTER_NONE;
  if (alt) {
    for (int i = 0; i < 8; i++)
      if (o.filter == kFilters[i]) filter = i;
    if (filter == MIP_FILTER_NONE) {
      std::cout << "  [!] ERROR: Filter type " << o.filter << " not supported" << std::endl;
      return 0;  // main.cpp:74-76 exits with 0
    }
  }
  if (errors > 0) {
    std::cout << "Exiting after finding errors in input parameters" << std::endl;
    return 1;
  }
  int W = 0, H = 0;
  if (sscanf(o.resolution.c_str(), "%dx%d", &W, &H) != 2 || W <= 0 || H <= 0) {
    std::cout << "  [!] ERROR: Input resolution \"" << o.resolution << "\" not set properly" << std::endl;
    return 0;
  }
  // The reference's resolution table (constants.h:17-23, main.cpp:301-309).  This engine also
  // takes every other size that is a multiple of 4 unless --StrictResolution is given.
  static const int kRefRes[5][2] = {{3840, 2160}, {1920, 1080}, {1280, 720}, {832, 480}, {416, 240}};
  bool listed = false;
  for (const auto &r : kRefRes) listed = listed || (r[0] == W && r[1] == H);
  if ((o.strict_res && !listed) || W % 4 || H % 4) {
    printf("[!] ERROR: Unsupported resolution %dx%d\n", W, H);
    printf("Supported resolutions are:\n");
    for (const auto &r : kRefRes) printf("  %dx%d\n", r[0], r[1]);
    if (!o.strict_res) printf("  (and any other width x height that are multiples of 4)\n");
    return 0;
  }
  const std::string fmt = input_format(o);
  const int threads = o.threads > 0 ? o.threads : (int)std::max(1u, std::thread::hardware_concurrency());
  FrameSource src;
  if (!src.open(o.input, fmt, W, H, threads)) {
    perror("error while opening samples files");
    return 1;
  }
  const int nctus = mip_num_ctus(W, H);
  mip_opts opts;
  mip_opts_default(&opts);
  opts.filter = filter;
  opts.kernel_idx = o.kernel_idx;
  // Frames per device batch: each batch is one synchronous mip_search_frames call, whose
  // pipeline fill and drain (first upload, last download) are paid per batch -- 8-frame
  // batches searched 64 1080p frames in 23 ms, the search itself takes ~8.5 ms.  Auto: about
  // 256 MB of samples per batch (32 frames at 1080p, 3 at 8K), bounding the pinned slots.
  const int auto_batch = (int)std::max<long long>(1, std::min<long long>(32, (256LL << 20) / ((long long)W * H * 2)));
  opts.max_batch = std::min(o.batch > 0 ? o.batch : auto_batch, std::max(1, o.frames));
  opts.want_sad_satd = o.sad_satd ? 1 : 0;
  opts.best_k = o.topk;
  std::vector<mip_engine *> engines;
  auto destroy_all = [&]() {
    for (mip_engine *e : engines) mip_engine_destroy(e);
    engines.clear();
  };
  for (int dev : o.devices) {
    mip_engine *e = nullptr;
    if (mip_engine_create(dev, W, H, &opts, &e) != 0) {
      std::cout << "  [!] ERROR: " << mip_last_error() << std::endl;
      destroy_all();
      return 1;
    }
    engines.push_back(e);
    if (filter != MIP_FILTER_NONE && mip_trace_times(e, 1) != 0) {
      std::cout << "  [!] ERROR: " << mip_last_error() << std::endl;
      destroy_all();
      return 1;
    }
  }
  const int ndev = (int)engines.size();
  const size_t fs = (size_t)W * H;
  const size_t cpf = (size_t)nctus * MIP_COSTS_PER_CTU_ABI, upf = (size_t)nctus * MIP_CUS_PER_CTU_ABI * o.topk;
  const int nlog = o.all_frames ? o.frames : std::min(1, o.frames);
  const bool want_best = !o.best_modes.empty(), want_bin = !o.binary_log.empty();

  std::vector<ShapeInfo> shapes(47);
  for (int s = 0; s < 47; s++) {
    ShapeInfo &sh = shapes[s];
    mip_shape_info(s, &sh.w, &sh.h, &sh.modes, &sh.ncu, &sh.off);
    sh.name = mip_shape_name(s);
    sh.x.resize(sh.ncu);
    sh.y.resize(sh.ncu);
    for (int cu = 0; cu < sh.ncu; cu++) mip_cu_position(s, cu, &sh.x[cu], &sh.y[cu]);
  }
  // Output files.  reportDistortionToFile=1 in the reference even when -l is not given
  // (writes ".csv").  Binary log header: "MIPC", version 1, width, height, frames, entries
  // per frame, flags (bit 0: SAD and SATD tables follow the cost tables), reserved; then
  // int32 little-endian tables (costs of every frame, then SAD, then SATD).
  FILE *log_fp = fopen((o.prefix + ".csv").c_str(), "w");
  if (!log_fp) { perror("cannot open cost log"); destroy_all(); return 1; }
  fprintf(log_fp, "CTU,cuSizeName,W,H,CU,X,Y,Mode,SAD,SATD,minSadHad\n");
  FILE *best_fp = nullptr, *bin_fp = nullptr;
  if (want_best) {
    best_fp = fopen(o.best_modes.c_str(), "w");
    if (!best_fp) { perror("cannot open best-mode file"); destroy_all(); return 1; }
    if (o.topk == 1) fprintf(best_fp, "Frame,CTU,cuSizeName,W,H,CU,X,Y,BestMode,Transposed,Cost\n");
    else fprintf(best_fp, "Frame,CTU,cuSizeName,W,H,CU,X,Y,Rank,Mode,Transposed,Cost\n");
  }
  if (want_bin) {
    bin_fp = fopen(o.binary_log.c_str(), "wb");
    if (!bin_fp) { perror("cannot open binary log"); destroy_all(); return 1; }
    const uint32_t hdr[8] = {0x4350494du, 1u, (uint32_t)W, (uint32_t)H, (uint32_t)o.frames, (uint32_t)cpf,
                             o.sad_satd ? 1u : 0u, 0u};
    if (fwrite(hdr, 4, 8, bin_fp) != 8) { perror("writing binary log"); destroy_all(); return 1; }
  }

  // Chunk pipeline over kSlots buffer slots: a reader thread fills a slot's frames, this
  // thread searches them (frames sharded over the engines, one host thread per device),
  // a writer thread emits the chunk's log rows / decision rows / binary tables in frame
  // order and frees the slot.  Host memory is bounded by kSlots chunks.
  constexpr int kSlots = 3;
  const int chunk = std::max(1, opts.max_batch) * ndev;
  const int nchunks = o.frames > 0 ? (o.frames + chunk - 1) / chunk : 0;
  struct Slot {
    Pinned<uint16_t> in;
    Pinned<int32_t> cost, sad, satd, best_cost;
    Pinned<uint8_t> best;
    int state = 0;  // 0 free, 1 frames read, 2 searched
  };
  std::vector<Slot> slots(kSlots);
  const bool cost_all = want_bin || o.all_frames;
  bool ok = true;
  const int near = ndev == 1 ? o.devices[0] : -1;  // (a slot's frames are shared by every device's shard)
  for (Slot &sl : slots) {
    const size_t n = (size_t)std::min(chunk, std::max(1, o.frames));
    ok = ok && sl.in.alloc(n * fs, near) && sl.cost.alloc((cost_all ? n : 1) * cpf, near);
    if (o.sad_satd)
      ok = ok && sl.sad.alloc((cost_all ? n : 1) * cpf, near) && sl.satd.alloc((cost_all ? n : 1) * cpf, near);
    if (want_best) ok = ok && sl.best.alloc(n * upf, near) && sl.best_cost.alloc(n * upf, near);
  }
  if (!ok) {
    std::cout << "  [!] ERROR: " << mip_last_error() << std::endl;
    destroy_all();
    return 1;
  }
  std::mutex mu;
  std::condition_variable cv;
  bool read_failed = false, search_failed = false, write_failed = false;
  auto wait_state = [&](int s, int st) {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return slots[s].state == st || read_failed || search_failed || write_failed; });
    return slots[s].state == st;
  };
  auto set_state = [&](int s, int st) {
    { std::lock_guard<std::mutex> lk(mu); slots[s].state = st; }
    cv.notify_all();
  };
  auto fail = [&](bool &flag) {
    { std::lock_guard<std::mutex> lk(mu); flag = true; }
    cv.notify_all();
  };
  auto chunk_range = [&](int c, int &f0, int &n) { f0 = c * chunk; n = std::min(chunk, o.frames - f0); };

  std::thread reader([&] {
    for (int c = 0; c < nchunks; c++) {
      const int s = c % kSlots;
      if (!wait_state(s, 0)) return;
      int f0, n;
      chunk_range(c, f0, n);
      if (!src.read(n, slots[s].in.data())) return fail(read_failed);
      set_state(s, 1);
    }
  });
  const int ctu_cols = (W + 127) / 128;
  std::thread writer([&] {
    for (int c = 0; c < nchunks; c++) {
      const int s = c % kSlots;
      if (!wait_state(s, 2)) return;
      Slot &sl = slots[s];
      int f0, n;
      chunk_range(c, f0, n);
      bool wok = true;
      for (int i = 0; i < n; i++) {
        const int f = f0 + i;
        const size_t co = cost_all ? i * cpf : 0;  // slot-local cost table of frame f
        if (f < nlog)
          write_cost_log(log_fp, shapes, nctus, W, sl.cost.data() + co, o.sad_satd ? sl.sad.data() + co : nullptr,
                         o.sad_satd ? sl.satd.data() + co : nullptr, threads);
        if (want_bin) {
          const long long base = 32, tab = (long long)cpf * 4;
          wok = wok && fseeko(bin_fp, base + f * tab, SEEK_SET) == 0 && fwrite(sl.cost.data() + co, 4, cpf, bin_fp) == cpf;
          if (o.sad_satd)
            wok = wok && fseeko(bin_fp, base + (o.frames + f) * tab, SEEK_SET) == 0 &&
                  fwrite(sl.sad.data() + co, 4, cpf, bin_fp) == cpf &&
                  fseeko(bin_fp, base + (2LL * o.frames + f) * tab, SEEK_SET) == 0 &&
                  fwrite(sl.satd.data() + co, 4, cpf, bin_fp) == cpf;
        }
        if (want_best)
          write_best_rows(best_fp, shapes, nctus, ctu_cols, f, o.topk, sl.best.data() + i * upf,
                          sl.best_cost.data() + i * upf, threads);
      }
      if (!wok) return fail(write_failed);
      set_state(s, 0);
    }
  });

  // "Elapsed time from writing samples to reading distortion" (main_aux_functions.h:192-211,
  // 908-914): the summed wall time of the chunks' device round trips (H2D, search, D2H);
  // file reading and log writing, outside that window in the reference, overlap it here.
  std::chrono::steady_clock::duration search_time{};
  double write_ns = 0;  // the reference's writeTime_filter
  std::vector<int> rcs(ndev, 0);
  std::vector<std::string> errs(ndev);
  for (int c = 0; c < nchunks && !search_failed; c++) {
    const int s = c % kSlots;
    if (!wait_state(s, 1)) break;
    Slot &sl = slots[s];
    int f0, n;
    chunk_range(c, f0, n);
    const bool need_cost = cost_all || f0 < nlog;
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> workers;
    for (int d = 0; d < ndev; d++) {
      const int a = (int)((long long)n * d / ndev), b = (int)((long long)n * (d + 1) / ndev);
      if (b <= a) continue;
      // costs: every frame when all are logged / binary-logged, else only the chunk's
      // first frame (frame 0, the reference's log) and only for the engine that has it
      const bool dc = need_cost && (cost_all || a == 0);
      const size_t co = cost_all ? a * cpf : 0;
      const int nb = cost_all || !dc ? b - a : 1;
      workers.emplace_back([&, d, a, b, dc, co, nb] {
        (void)mip_bind_thread(o.devices[d]);  // the device's host thread on its GPU's NUMA node
        rcs[d] = 0;
        if (!dc || nb == b - a)
          rcs[d] = mip_search_frames(engines[d], sl.in.data() + a * fs, nullptr, b - a, dc ? sl.cost.data() + co : nullptr,
                                     want_best ? sl.best.data() + a * upf : nullptr,
                                     want_best ? sl.best_cost.data() + a * upf : nullptr,
                                     dc && o.sad_satd ? sl.sad.data() + co : nullptr,
                                     dc && o.sad_satd ? sl.satd.data() + co : nullptr);
        else  // the first frame's tables, then the rest without tables
          rcs[d] = mip_search_frames(engines[d], sl.in.data() + a * fs, nullptr, 1, sl.cost.data(),
                                     want_best ? sl.best.data() + a * upf : nullptr,
                                     want_best ? sl.best_cost.data() + a * upf : nullptr,
                                     o.sad_satd ? sl.sad.data() : nullptr, o.sad_satd ? sl.satd.data() : nullptr) ||
                   (b - a > 1 &&
                    mip_search_frames(engines[d], sl.in.data() + (a + 1) * fs, nullptr, b - a - 1, nullptr,
                                      want_best ? sl.best.data() + (a + 1) * upf : nullptr,
                                      want_best ? sl.best_cost.data() + (a + 1) * upf : nullptr, nullptr, nullptr));
        if (rcs[d] != 0) errs[d] = mip_last_error();
      });
    }
    for (auto &w : workers) w.join();
    search_time += std::chrono::steady_clock::now() - t0;
    for (int d = 0; d < ndev; d++)
      if (rcs[d] != 0) {
        std::cout << "  [!] ERROR: device " << o.devices[d] << ": " << errs[d] << std::endl;
        fail(search_failed);
      }
    if (search_failed) break;
    // The reference's per-frame report (main.cpp:681, 709, 754, 771-775, 804, 911, 997,
    // 1076, 1153): the frame number, with alternative references the filter's device time,
    // and the stages -- boundaries, reduced prediction, upsampling + distortion -- which run
    // fused in one search launch here.
    std::vector<double> up_ms(n, 0.0), filt_ms(n, 0.0);
    if (filter != MIP_FILTER_NONE) {
      int got = 0;
      for (int d = 0; d < ndev; d++) {
        int k = 0;
        if (mip_pop_times(engines[d], up_ms.data() + got, filt_ms.data() + got, n - got, &k) == 0) got += k;
      }
      if (c == 0) write_ns = up_ms[0] * 1e6;  // writeTime_filter: the first frame's upload (main.cpp:580-595)
    }
    for (int i = 0; i < n; i++) {
      printf("Current frame %d\n", f0 + i);
      if (filter != MIP_FILTER_NONE) {
        const double exec_ns = filt_ms[i] * 1e6;
        printf("Performing filterFrame kernel...\n");
        printf("FilterSamples took %f ms\n\n", exec_ns / 1000000);
        printf("TIMING REPORT\n");
        printf("Write(ns): %f\n", write_ns);
        printf("Execution(ns):%f\n", exec_ns);
        printf("Read(ns): %f\n", 0.0);
        printf("TotalFilterTime(ms): %f\n", (write_ns + exec_ns) / 1000000);
      }
      printf("Performing initBoundaries kernel...\n");
      printf("Performing MIP_ReducedPred kernel...\n");
      for (int u = 0; u < 3; u++) printf("Performing upsampleDistortion kernel...\n");
    }
    fflush(stdout);
    set_state(s, 2);
  }
  reader.join();
  writer.join();
  fclose(log_fp);
  if (best_fp) fclose(best_fp);
  const bool bin_ok = !bin_fp || fclose(bin_fp) == 0;
  if (read_failed && src.range_error() >= 0) {
    const long long b = src.range_error(), fs1 = (long long)W * H;
    std::cout << "  [!] ERROR: input sample " << b / fs1 << ":" << (b % fs1) / W << ":" << b % W
              << " (frame:row:column) is above 10 bits (> 1023); samples must be 10-bit values" << std::endl;
    destroy_all();
    return 1;
  }
  if (read_failed) {
    perror("error while opening samples files");
    destroy_all();
    return 1;
  }
  if (search_failed) { destroy_all(); return 1; }
  if (write_failed || !bin_ok) { perror("writing binary log"); destroy_all(); return 1; }
  const long ms = (long)std::chrono::duration_cast<std::chrono::milliseconds>(search_time).count();
  printf("=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=\n");
  printf("TIMING RESULTS (miliseconds)\n");
  printf("Elapsed time (ms) from writing samples to reading distortion (%dx), %ld\n", o.frames, ms);
  printf("=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=-=\n\n");
  destroy_all();
  return 0;
}
