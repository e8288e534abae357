// ffv1_host.cpp -- host side of the MI355X FFV1 encoder: the C-ABI of
// include/ffv1hip.h, encode_init's parameter contract, the (init-time)
// extradata writer, the per-slice header op lists and HBM buffer management.
// The per-sample work runs in ffv1_kernels.hip; nothing here touches pixels.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ffv1hip.h"
#include "ffv1_internal.h"

using namespace ffv1hip;

namespace {

thread_local char g_err[512];

int set_err(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

#define HIP_TRY(expr)                                                         \
  do {                                                                        \
    hipError_t e_ = (expr);                                                   \
    if (e_ != hipSuccess)                                                     \
      return set_err(-5, "%s failed: %s", #expr, hipGetErrorString(e_));      \
  } while (0)

// A few host threads for the copies between pageable caller memory and the
// pinned staging buffers of the host-frame path: run(fn) calls fn(part,
// nparts) on every worker and on the caller, and returns when all are done.
class CopyPool {
 public:
  explicit CopyPool(int n) : n_(std::max(1, n)) {
    for (int i = 1; i < n_; i++) th_.emplace_back([this, i] { loop(i); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (std::thread& t : th_) t.join();
  }
  int size() const { return n_; }
  void run(const std::function<void(int, int)>& fn) {
    if (n_ == 1) {
      fn(0, 1);
      return;
    }
    {
      std::lock_guard<std::mutex> g(m_);
      job_ = &fn;
      pending_ = n_ - 1;
      gen_++;
    }
    cv_.notify_all();
    fn(0, n_);
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [&] { return pending_ == 0; });
    job_ = nullptr;
  }

 private:
  void loop(int i) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int, int)>* job;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        job = job_;
      }
      (*job)(i, n_);
      std::lock_guard<std::mutex> g(m_);
      if (--pending_ == 0) done_.notify_one();
    }
  }
  int n_;
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void(int, int)>* job_ = nullptr;
  uint64_t gen_ = 0;
  int pending_ = 0;
  bool stop_ = false;
};

// Measurement and test hooks, all in one variable, read when a context is
// created (so each context sees the value set at its creation, and nothing is
// cached in function statics):
//   FFV1HIP_DEBUG="name[=value],name[=value],..."
// measurement: serial, walkdbg, walktrace, hostdbg, copy_threads, walk_prio,
// range_prio, sym_skip; test hooks (each forces a path the product takes on
// its own only in some configs or under memory pressure): coder=chain,
// dense=0, walk_blocks=0, recsets=1, slice_cap, walk_part_a, force_multi,
// bounds_shrink, dsets=eager|lazy, budget=q, rec2_drop=set, pack=0, fsets=2,
// v4_cap0, readback, guard_skip, compact=0, code_cpw=n.  Unknown names
// are an error at create time, so a misspelt hook never silently measures
// the default.
struct Knobs {
  std::vector<std::pair<std::string, std::string>> kv;
  const std::string* find(const char* name) const {
    for (const auto& e : kv)
      if (e.first == name) return &e.second;
    return nullptr;
  }
  bool has(const char* name) const { return find(name) != nullptr; }
  // "name" alone reads as 1
  int get(const char* name, int dflt) const {
    const std::string* v = find(name);
    return v ? (v->empty() ? 1 : std::atoi(v->c_str())) : dflt;
  }
  std::string str(const char* name) const {
    const std::string* v = find(name);
    return v ? *v : std::string();
  }
};

static const char* const kKnobNames[] = {"serial",      "walkdbg",     "walktrace", "hostdbg",       "copy_threads",
                                         "coder",       "dense",       "walk_blocks", "recsets",     "slice_cap",
                                         "walk_part_a", "force_multi", "bounds_shrink", "dsets",
                                         "rec2_drop",   "budget",      "pack",        "v4_cap0",     "readback",
                                         "fsets",       "guard_skip",  "walk_prio",   "range_prio",  "compact",
                                         "sym_skip",    "code_cpw"};

// The per-hook environment variables of earlier rounds.  They are no longer
// read, so one that is set is an error (a measurement that silently ran the
// default); every other FFV1HIP_* name (FFV1HIP_LIB, FFV1HIP_TWOPASS_LIB, ...)
// belongs to someone else and is left alone.
static const char* const kLegacyVars[] = {
    "FFV1HIP_BITS",          "FFV1HIP_BITS_INLINE", "FFV1HIP_CODEDBG",    "FFV1HIP_CODER",     "FFV1HIP_CODE_WAVE_PRIO",
    "FFV1HIP_COPYOUT_SYNC",  "FFV1HIP_COPY_THREADS", "FFV1HIP_DEC_SWAP",  "FFV1HIP_DENSE",     "FFV1HIP_FORCE_MULTI",
    "FFV1HIP_HOSTDBG",       "FFV1HIP_LANES",       "FFV1HIP_PARTIAL",    "FFV1HIP_RANGE_FAT", "FFV1HIP_RANGE_PRIO",
    "FFV1HIP_RECSETS",       "FFV1HIP_RESERVE_CUS", "FFV1HIP_SERIAL",     "FFV1HIP_SLICE_CAP", "FFV1HIP_SPLIT_MAX",
    "FFV1HIP_SYM_DELAY_US",  "FFV1HIP_WALKDBG",     "FFV1HIP_WALKTRACE",  "FFV1HIP_WALK_FAT",  "FFV1HIP_WALK_LDS_PAD",
    "FFV1HIP_WALK_LONG_BOOST", "FFV1HIP_WALK_PART_A", "FFV1HIP_WALK_PRIO", "FFV1HIP_WALK_SPLIT"};

static int parse_knobs(Knobs* k) {
  k->kv.clear();
  for (const char* name : kLegacyVars)
    if (std::getenv(name))
      return set_err(-22, "%s is not read: hooks go in FFV1HIP_DEBUG=name[=value],...", name);
  const char* e = std::getenv("FFV1HIP_DEBUG");
  if (!e) return 0;
  std::string all(e);
  size_t i = 0;
  while (i <= all.size()) {
    size_t j = all.find(',', i);
    if (j == std::string::npos) j = all.size();
    std::string item = all.substr(i, j - i);
    i = j + 1;
    if (item.empty()) continue;
    const size_t eq = item.find('=');
    std::string name = item.substr(0, eq), val = eq == std::string::npos ? "" : item.substr(eq + 1);
    bool known = false;
    for (const char* n : kKnobNames) known |= name == n;
    if (!known) return set_err(-22, "FFV1HIP_DEBUG: unknown hook '%s'", name.c_str());
    k->kv.emplace_back(name, val);
  }
  return 0;
}

double wall_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// rows of wb bytes from src (pitch sp) to dst (pitch dp), split over the pool
void pool_copy2d(CopyPool& pool, uint8_t* dst, int64_t dp, const uint8_t* src, int64_t sp, int64_t wb, int64_t rows) {
  if (rows <= 0 || wb <= 0) return;
  const bool flat = dp == wb && sp == wb;
  if (wb * rows < (int64_t(1) << 20) || pool.size() == 1) {
    if (flat) {
      std::memcpy(dst, src, size_t(wb * rows));
    } else {
      for (int64_t r = 0; r < rows; r++) std::memcpy(dst + r * dp, src + r * sp, size_t(wb));
    }
    return;
  }
  pool.run([&](int part, int np) {
    if (flat) {  // 4 KiB-aligned byte ranges
      const int64_t n = wb * rows, per = ((n + np - 1) / np + 4095) & ~int64_t(4095);
      const int64_t a = std::min(n, per * part), b = std::min(n, a + per);
      if (b > a) std::memcpy(dst + a, src + a, size_t(b - a));
    } else {
      const int64_t a = rows * part / np, b = rows * (part + 1) / np;
      for (int64_t r = a; r < b; r++) std::memcpy(dst + r * dp, src + r * sp, size_t(wb));
    }
  });
}

// Rows r0 .. r1-1 of w 16-bit samples (pitch sp bytes) packed three to a
// 32-bit word (bits 0-9, 10-19, 20-29) into rows of pb bytes at dst; returns
// the OR of the samples (>= 1024: they did not fit, the frame goes as is).
static uint32_t pack10_rows(uint8_t* dst, int64_t pb, const uint8_t* src, int64_t sp, int w, int64_t r0, int64_t r1) {
  uint32_t acc = 0;
  const int n3 = w / 3, tail = w - 3 * n3;
  for (int64_t r = r0; r < r1; r++) {
    const uint16_t* const s = reinterpret_cast<const uint16_t*>(src + r * sp);
    uint32_t* const d = reinterpret_cast<uint32_t*>(dst + r * pb);
    uint32_t m = 0;
    for (int j = 0; j < n3; j++) {
      const uint32_t a = s[3 * j], b = s[3 * j + 1], c = s[3 * j + 2];
      m |= a | b | c;
      d[j] = a | (b << 10) | (c << 20);
    }
    if (tail) {
      const uint32_t a = s[3 * n3], b = tail == 2 ? s[3 * n3 + 1] : 0u;
      m |= a | b;
      d[n3] = a | (b << 10);
    }
    acc |= m;
  }
  return acc;
}

static uint32_t pool_pack10(CopyPool& pool, uint8_t* dst, int64_t pb, const uint8_t* src, int64_t sp, int w,
                            int64_t rows) {
  if (rows <= 0) return 0;
  if (int64_t(w) * 2 * rows < (int64_t(1) << 20) || pool.size() == 1) return pack10_rows(dst, pb, src, sp, w, 0, rows);
  std::atomic<uint32_t> acc{0};
  pool.run([&](int part, int np) {
    acc.fetch_or(pack10_rows(dst, pb, src, sp, w, rows * part / np, rows * (part + 1) / np));
  });
  return acc.load();
}

// ---------------------------------------------------------------------------
// Transition tables.  Default: ff_build_rac_states(c, 0.05*2^32, 256-8)
// (rangecoder.c:63-101); custom: the FFV1 v2+ table (ffv1enc.c:120-137)
// installed as in ffv1.c:95-101.
struct Tables {
  uint8_t to0[256], to1[256];
};

Tables default_tables() {
  Tables t;
  std::memset(&t, 0, sizeof(t));
  const int64_t one = int64_t(1) << 32;
  const int factor = int(0.05 * double(int64_t(1) << 32));
  const int max_p = 248;
  int64_t p = one / 2;
  int last = 0;
  for (int i = 0; i < 128; i++) {
    int p8 = int((256 * p + one / 2) >> 32);
    if (p8 <= last) p8 = last + 1;
    if (last && last < 256 && p8 <= max_p) t.to1[last] = uint8_t(p8);
    p += ((one - p) * factor + one / 2) >> 32;
    last = p8;
  }
  for (int i = 256 - max_p; i <= max_p; i++) {
    if (t.to1[i]) continue;
    int64_t q = (int64_t(i) * one + 128) >> 8;
    q += ((one - q) * factor + one / 2) >> 32;
    int p8 = int((256 * q + one / 2) >> 32);
    if (p8 <= i) p8 = i + 1;
    if (p8 > max_p) p8 = max_p;
    t.to1[i] = uint8_t(p8);
  }
  for (int i = 1; i < 255; i++) t.to0[i] = uint8_t(256 - t.to1[256 - i]);
  return t;
}

const uint8_t kCustomStt[256] = {
    0,   10,  10,  10,  10,  16,  16,  16,  28,  16,  16,  29,  42,  49,  20,  49,
    59,  25,  26,  26,  27,  31,  33,  33,  33,  34,  34,  37,  67,  38,  39,  39,
    40,  40,  41,  79,  43,  44,  45,  45,  48,  48,  64,  50,  51,  52,  88,  52,
    53,  74,  55,  57,  58,  58,  74,  60,  101, 61,  62,  84,  66,  66,  68,  69,
    87,  82,  71,  97,  73,  73,  82,  75,  111, 77,  94,  78,  87,  81,  83,  97,
    85,  83,  94,  86,  99,  89,  90,  99,  111, 92,  93,  134, 95,  98,  105, 98,
    105, 110, 102, 108, 102, 118, 103, 106, 106, 113, 109, 112, 114, 112, 116, 125,
    115, 116, 117, 117, 126, 119, 125, 121, 121, 123, 145, 124, 126, 131, 127, 129,
    165, 130, 132, 138, 133, 135, 145, 136, 137, 139, 146, 141, 143, 142, 144, 148,
    147, 155, 151, 149, 151, 150, 152, 157, 153, 154, 156, 168, 158, 162, 161, 160,
    172, 163, 169, 164, 166, 184, 167, 170, 177, 174, 171, 173, 182, 176, 180, 178,
    175, 189, 179, 181, 186, 183, 192, 185, 200, 187, 191, 188, 190, 197, 193, 196,
    197, 194, 195, 196, 198, 202, 199, 201, 210, 203, 207, 204, 205, 206, 208, 214,
    209, 211, 221, 212, 213, 215, 224, 216, 217, 218, 219, 220, 222, 228, 223, 225,
    226, 224, 227, 229, 240, 230, 231, 232, 233, 234, 235, 236, 238, 239, 237, 242,
    241, 243, 242, 244, 245, 246, 247, 248, 249, 250, 251, 252, 252, 253, 254, 255,
};

Tables custom_tables(const Tables& dflt) {
  Tables t = dflt;
  for (int i = 1; i < 256; i++) {
    t.to1[i] = kCustomStt[i];
    t.to0[256 - i] = uint8_t(256 - kCustomStt[i]);
  }
  return t;
}

// ---------------------------------------------------------------------------
// Quantisation tables (ffv1enc.c:44-118, 846-879), expressed by the first
// index of each quantiser step on [0,127]; the negative half mirrors.
void quant_table(int16_t* q, std::initializer_list<int> steps, int scale) {
  int level = 0;
  auto it = steps.begin();
  for (int i = 0; i < 128; i++) {
    while (it != steps.end() && i >= *it) { ++level; ++it; }
    q[i] = int16_t(scale * level);
  }
  for (int i = 1; i < 128; i++) q[256 - i] = int16_t(-q[i]);
  q[128] = int16_t(-q[127]);
}

void quant_set(int16_t qt[5][256], int model, int bits) {
  std::memset(qt, 0, sizeof(int16_t) * 5 * 256);
  const bool hi = bits > 8;
  auto A = hi ? std::initializer_list<int>{5, 13, 27, 56} : std::initializer_list<int>{1, 2, 5, 12, 35};
  auto B = hi ? std::initializer_list<int>{11, 50} : std::initializer_list<int>{1, 4};
  quant_table(qt[0], A, 1);
  quant_table(qt[1], A, 11);
  if (model == 0) {
    quant_table(qt[2], A, 121);
  } else {
    quant_table(qt[2], B, 121);
    quant_table(qt[3], B, 605);
    quant_table(qt[4], B, 3025);
  }
}

int contexts_of(int model) { return model ? (11 * 11 * 5 * 5 * 5 + 1) / 2 : (11 * 11 * 11 + 1) / 2; }

// ---------------------------------------------------------------------------
// Host range coder: only for the init-time extradata (write_extradata is
// host work in the reference too, ffv1enc.c:545-619).
struct HostRac {
  int low = 0, range = 0xFF00, pending = -1, run = 0;
  std::vector<uint8_t> out;
  const Tables* t;
  explicit HostRac(const Tables* tab) : t(tab) {}
  void shift() {
    while (range < 0x100) {
      if (pending < 0) {
        pending = low >> 8;
      } else if (low <= 0xFF00) {
        out.push_back(uint8_t(pending));
        for (; run; run--) out.push_back(0xFF);
        pending = low >> 8;
      } else if (low >= 0x10000) {
        out.push_back(uint8_t(pending + 1));
        for (; run; run--) out.push_back(0x00);
        pending = (low >> 8) & 0xFF;
      } else {
        run++;
      }
      low = (low & 0xFF) << 8;
      range <<= 8;
    }
  }
  void put(uint8_t* st, int bit) {
    int r1 = (range * *st) >> 8;
    if (bit) { low += range - r1; range = r1; *st = t->to1[*st]; }
    else { range -= r1; *st = t->to0[*st]; }
    shift();
  }
  void symbol(uint8_t* st, int v, bool sgn) {
    if (!v) { put(st, 1); return; }
    unsigned a = v < 0 ? 0u - unsigned(v) : unsigned(v);
    int e = 31 - __builtin_clz(a);
    put(st, 0);
    for (int i = 0; i < e; i++) put(st + 1 + std::min(i, 9), 1);
    put(st + 1 + std::min(e, 9), 0);
    for (int i = e - 1; i >= 0; i--) put(st + 22 + std::min(i, 9), (a >> i) & 1);
    if (sgn) put(st + 11 + std::min(e, 10), v < 0);
  }
  void finish() {
    range = 0xFF; low += 0xFF; shift();
    range = 0xFF; shift();
  }
};

uint32_t crc32_msb(const uint8_t* p, size_t n) {
  uint32_t crc = 0;
  for (size_t i = 0; i < n; i++) {
    crc ^= uint32_t(p[i]) << 24;
    for (int k = 0; k < 8; k++) crc = (crc & 0x80000000u) ? (crc << 1) ^ 0x04C11DB7u : (crc << 1);
  }
  return crc;
}

// Table-driven form of crc32_msb (av_crc with AV_CRC_32_IEEE,
// libavutil/crc.c:356-380), for the decoder's slice checks.
uint32_t crc32_msb_fast(const uint8_t* p, size_t n) {
  static const std::vector<uint32_t> tab = [] {
    std::vector<uint32_t> t(256);
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i << 24;
      for (int k = 0; k < 8; k++) c = (c & 0x80000000u) ? (c << 1) ^ 0x04C11DB7u : (c << 1);
      t[i] = c;
    }
    return t;
  }();
  uint32_t crc = 0;
  for (size_t i = 0; i < n; i++) crc = (crc << 8) ^ tab[(crc >> 24) ^ p[i]];
  return crc;
}

// Recorder used to turn a header writer into an op list for the device.
struct OpList {
  std::vector<Op> ops;
  void sym(int set, int tab, int v, bool sgn) { ops.push_back(Op{int16_t(sgn ? kOpSymS : kOpSymU), uint8_t(set), uint8_t(tab), v}); }
  void bit(int set, int tab, int v) { ops.push_back(Op{int16_t(kOpBit), uint8_t(set), uint8_t(tab), v}); }
};

}  // namespace

// ---------------------------------------------------------------------------
struct ffv1hip_ctx {
  Knobs knobs;  // FFV1HIP_DEBUG at create time
  ffv1hip_params P{};
  int device = 0;
  int max_batch = 0;
  int nslices = 0;
  int contexts = 0;
  Tables dflt{}, frame{};
  int16_t qt[5][256]{};
  std::vector<uint8_t> extradata;
  std::vector<Op> ops;     // [key][slice][kMaxOps]
  std::vector<int> nops;   // [key][slice]
  int64_t slice_cap = 0;
  int64_t slice_stride = 0;  // bytes per slice slot of d_slice_out
  int64_t packet_stride = 0;
  int64_t frame_bytes = 0;  // host-layout batch buffer stride
  int64_t plane_bytes[kMaxPlanes]{};  // input planes of a frame slot (YUVA: Y, Cb, Cr, A)
  int pcount = 2;                     // plane contexts: plane_count, 2 + transparency (ffv1enc.c:720, 890-891)
  int ncoded = 3;                     // coded planes of a slice (symbols kernel z, chained coders)
  int64_t picture_number = 0;
  bool have_states = false;  // persistent states valid (a frame was coded)
  int max_slots = 0;          // segments (= frame slots) per call
  bool frames_mode = false;   // states walk + decision-stream coder (range coder, LDS-sized tables)
  int wmax = 0;               // most decisions one symbol can take (2 * coded bits + 1)
  int cwords = kChunkWords;   // frames mode: words per walk chunk (chunk_words(wmax))
  int64_t batches_run = 0;    // frames-mode batches started (the sym_skip measurement hook)
  int64_t table_dummy = 0;    // chained mode: the first of ffv1_code's dummy tables
  int64_t frame_samples = 0;  // symbols of one frame (each slice padded to 4)
  int64_t frame_chunks = 0;   // 64-sample walk chunks of one frame
  int max_ops = 0;
  std::vector<SliceGeom> geom;
  // device buffers
  uint8_t* d_frames = nullptr;
  int16_t* d_qt = nullptr;
  int walk_rows = 0;             // frames mode: context rows per plane group in the walk's LDS
  int walk_rowb = 32;            // ... and bytes per row (kCompactRowBytes at 8 bits)
  int16_t* d_qt_walk = nullptr;  // dense rows (kDenseRows): quant tables with weights 1, 9, 81
  uint8_t* d_tabs = nullptr;
  Op* d_ops = nullptr;
  int* d_nops = nullptr;
  Segment* d_segs = nullptr;
  uint8_t* d_keys = nullptr;
  uint8_t* d_slice_out = nullptr;
  int64_t* d_slice_bytes = nullptr;
  uint8_t* d_packets = nullptr;
  int64_t* d_packet_size = nullptr;
  // the P-frame carry, [slice][2][contexts][32], double-buffered: a batch
  // reads d_persist[pcur] and writes d_persist[pcur ^ 1] (its segments may
  // load and save the same slice in one launch, in any block order)
  uint8_t* d_persist[2] = {nullptr, nullptr};
  int pcur = 0;
  uint8_t* d_tables = nullptr;   // [slot][slice][2][contexts][32]
  uint32_t* d_sym = nullptr;     // [slot][frame_samples]; frames mode: walk records (uint2), set 0 of [batch frame][frame_samples]
  // frames mode, two buffer sets: the walk of batch k+1 runs while batch k codes
  uint8_t* d_keys2 = nullptr;    // 3 x [batch frame] keyflags
  uint32_t* d_cbits = nullptr;   // 2 x [batch frame][frame_chunks][cwords] packed decision bits
  // the per-batch stream metadata has three sets (index tri): the symbols of
  // batch k rewrite set k % 3 while the coder of batch k-1 may still read its
  // set and the walk of batch k-1 run
  int* d_dcount = nullptr;       // 3 x [batch frame][slice][3] decisions per plane
  int64_t* d_dbase = nullptr;    // 3 x [batch frame][slice] first decision of each stream
  int64_t* d_dtotal = nullptr;   // [3] decisions of the batch (incl. alignment)
  int64_t* h_dtotal = nullptr;   // pinned readback of d_dtotal
  // the totals as the layout kernels leave them, in mapped host memory, and
  // the frames of the batch in each metadata set: the estimate that lets a
  // batch launch without waiting for its own total (a guarded launch)
  int64_t* h_tot_map = nullptr;
  int64_t* hd_tot_map = nullptr;
  int tri_n[3] = {0, 0, 0};
  bool no_guard_once = false;    // the next run_batch sizes its set from the read-back total
  int64_t guard_skips = 0;       // batches the guard_skip hook launched to be skipped (ffv1hip_debug_counter)
  int64_t guard_reruns = 0;      // guarded batches encoded again at settle (status[3])
  uint8_t* d_pre[2] = {nullptr, nullptr};    // [decision] state before the decision
  uint8_t* d_scratch = nullptr;               // where idle walk chains write their stage
  uint32_t* d_bounds = nullptr;               // debug build: the first out-of-bounds write's site (sticky)
  uint32_t* d_bits[2] = {nullptr, nullptr};  // [decision / 32] decision bits
  // the three-pass coder (ffv1_range / ffv1_dseg / ffv1_dfix): the header's
  // digits per (key, slice), the per-stream segment layout (three sets, with
  // the stream metadata), checkpoints and segment records (one set: only
  // the coder stream uses them)
  HdrState* d_hdr = nullptr;
  uint32_t* d_hdr_digits = nullptr;
  std::vector<HdrState> hdr;
  std::vector<uint32_t> hdr_digits;
  StreamSegs* d_segs_info = nullptr;  // 3 x [batch frame][slice]
  int* d_seg_totals = nullptr;        // 3 x [2]
  int* d_wmap = nullptr;              // 3 x [64-segment group]
  int64_t max_groups = 0;             // 64-segment groups a batch can have
  int64_t max_segs = 0;               // segments a batch can have
  uint2* d_ck = nullptr;
  uint2* d_segrec = nullptr;
  int2* d_rstate = nullptr;  // [stream] the range pass's {range, shifts} at the luma / chroma boundary
  int64_t dcap[2] = {0, 0};      // decisions d_pre/d_bits hold
  int buf = 0;                   // buffer set of the next batch
  hipStream_t code_stream = nullptr;  // ffv1_range .. assembly, behind the states walk
  hipEvent_t walked[2] = {nullptr, nullptr};
  hipStream_t bits_stream = nullptr;  // ffv1_bits, beside the states walk
  hipEvent_t laid[2] = {nullptr, nullptr};    // set k's stream layout and zeroed bits are ready
  hipEvent_t bitsed[2] = {nullptr, nullptr};  // set k's decision bits are in place
  hipEvent_t coded[2] = {nullptr, nullptr};  // the coder of the batch that last used set k is done
  hipEvent_t pre_read[2] = {nullptr, nullptr};  // ... has read its decision stream (range, dseg): set k is free
  int tri = 0;                                // metadata set of the next batch
  hipEvent_t coded3[3] = {nullptr, nullptr, nullptr};  // the coder of the batch that last used metadata set k
  // Split schedule (a second set of walk records and chunk bits, when HBM
  // allows): the walk is launched in two parts, first the waves the CUs hold
  // at once (the long plane group's chains and some of the short), then the
  // rest; the symbols, layout and bits of batch k+1 run on the bits stream
  // once the first part of batch k's walk is done, beside its second part,
  // instead of in front of the next walk on its stream
  bool two_rec = false;
  uint2* d_rec2 = nullptr;       // [batch frame][frame_samples] walk records of set 1
  uint32_t* d_cbits2 = nullptr;  // chunk bits of set 1
  // the decision sets of a large batch are sized from the first batches'
  // decisions (lazy), and the second records set is taken from what they
  // leave (rec2_pending until the first batch has sized set 0)
  bool lazy_sets = false;
  bool rec2_pending = false;
  int* d_ident = nullptr;        // [batch frame] i: the frames mode's frame of each slot
  hipEvent_t entry[2] = {nullptr, nullptr};  // set k's batch: the launch stream's work so far
  hipEvent_t xchg_ev = nullptr;               // ffv1hip_set_slice_states_device: the caller's stream so far
  hipEvent_t walk_a = nullptr;               // the first part of the last batch's walk is done
  hipEvent_t walk_go = nullptr;              // everything before the last batch's walk is done (it starts)
  bool walk_a_valid = false;
  // grid caps of the kernels that run beside the states walk (their blocks
  // stride over the work): a grid of one block per item fills every SIMD's
  // wave slots and registers, and walk waves launched meanwhile wait for CU
  // room until those blocks retire (values measured best in earlier rounds)
  int grid_sym = 4096, grid_bits = 2048, grid_dseg = 4096;
  int cus = 256;      // compute units of the device (a walk wave per SIMD: 4 per CU)
  int lds_block = 0;  // LDS one workgroup may take (the walk's 4/5-wave blocks are held to it)
  int prio_dseg = 0;  // dseg's wave priority (walk / range: per batch, run_batch)
  SliceGeom* d_geom = nullptr;
  int* d_slot_frames = nullptr;  // [j][slot]
  int* d_status = nullptr;       // [set][4]: [0] slices over budget, [1] most bytes one needed
  int2* d_rct = nullptr;         // v4: [batch frame][slice] RCT coefficients (choose_rct_params)
  hipStream_t stream = nullptr;
  // 2-pass (ffv1enc.c:898-986): pass 1 counts into d_rcstat ([256][2] state
  // counts, then [contexts][32][2] slot counts); pass 2 starts keyframes
  // from init_states[context_model] (d_init)
  int pass = 0;
  unsigned long long* d_rcstat = nullptr;
  unsigned long long* d_rcstat_bak = nullptr;  // before the last batch (its re-encode)
  int64_t gob_count = 0;                       // keyframes coded (ffv1enc.c:1302)
  std::vector<uint8_t> init_states[2];
  uint8_t* d_init = nullptr;
  // ordering between calls: the next batch's launch stream waits for `dep`
  // (the previous batch's last use of the buffers it rewrites first), and
  // ffv1hip_synchronize waits for `done` (the previous batch's last kernel)
  hipEvent_t dep_ev = nullptr, done_ev = nullptr;
  bool dep_valid = false;
  // The last two batches (slot b & 1 for batch b), kept so that a slice over
  // the byte budget can be encoded again with a larger budget
  // (settle_batch): the inputs, and the state before the batch.
  struct LastBatch {
    bool valid = false;
    const uint8_t* frames = nullptr;
    int64_t frame_bytes = 0;
    int64_t plane_off[kMaxPlanes]{};
    int plane_stride[kMaxPlanes]{};
    int n = 0;
    hipStream_t st = nullptr;
    int64_t pn0 = 0;
    bool have0 = false;
    int pcur0 = 0, buf0 = 0, tri0 = 0, pk0 = 0, status_set = 0;
    int pk = 0;  // the packet set its packets are in
    int64_t gob0 = 0;
    std::vector<int> keys;
  } hist[2];
  hipEvent_t hist_done[2] = {nullptr, nullptr};  // batch slot k's last kernel
  // FFV1HIP_DEBUG=walktrace (measurement hook): every walk wave's start and end
  // (s_memrealtime, 100 MHz) for up to kTraceBatches batches, kept on the
  // device and summarised at ffv1hip_destroy: dispatch spread and duration
  // of each launch part
  static constexpr int kTraceBatches = 64;
  uint64_t* d_trace = nullptr;
  int trace_items = 0, trace_n = 0;
  std::vector<int> trace_first;  // per traced batch: part A's waves (0: one launch)
  int64_t nsub = 0;                              // batches submitted
  // packet slots: set 0 always; a second set (two_pk) for the host-frame
  // path, so that batch k's packets are copied out while batch k+1 codes
  uint8_t* d_packets2 = nullptr;
  int64_t* d_packet_size2 = nullptr;
  bool two_pk = false;
  int pk = 0;  // packet set of the next batch
  uint8_t* pkts(int set) const { return set ? d_packets2 : d_packets; }
  int64_t* psize(int set) const { return set ? d_packet_size2 : d_packet_size; }
  const LastBatch& last() const { return hist[(nsub + 1) & 1]; }
  bool profiling = false;
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
  std::vector<hipEvent_t> kev;  // [2 * launches]: start/stop per kernel launch
  std::vector<int> kev_kind;    // per launch: 0 symbols, 1 code (ffv1_range), 2 states, 3 assembly, 4 layout,
                                // 5 bits, 6 sink, 7 dseg, 8 dfix
  int nkev = 0;
  int last_nsegs = 0;
  // ffv1hip_encode2 (AV_CODEC_CAP_DELAY): frames queued in d_frames slots
  // 0..q_pts.size()-1, and encoded packets not yet handed out
  std::vector<int64_t> q_pts;
  struct Ready {
    const uint8_t* base = nullptr;  // the pinned packets of its packet set
    std::vector<int64_t> off, size, pts;
    std::vector<int> key;
    size_t next = 0;
  } ready;
  // The host-frame path (ffv1hip_encode / ffv1hip_encode2): frames are
  // copied in through pinned staging slots by the pool's threads, on a
  // transfer stream of its own, into one of two frame sets (d_frames,
  // d_frames2); packets come back through a pinned buffer per packet set.
  struct HostPipe {
    bool on = false;
    bool overlap = false;  // two frame sets and two packet sets: batch k+1 stages while batch k codes
    // frame sets: 1, 2 (overlap) or 3 (ffv1hip_encode stages batch k+2
    // while batch k finishes, collecting it only before k+2's launch)
    int nsets = 1;
    std::unique_ptr<CopyPool> pool;
    std::unique_ptr<CopyPool> pool_out;  // the copy-out thread's: packets into the caller's buffer
    hipStream_t xfer = nullptr;
    hipStream_t d2h = nullptr;  // ffv1hip_encode: packets out beside the next batch's frames in
    static constexpr int kSlots = 6;
    int64_t slot_bytes = 0;
    uint8_t* h_slot[kSlots]{};
    hipEvent_t slot_ev[kSlots]{};
    bool slot_busy[kSlots]{};
    int next = 0;
    int64_t fill = 0;
    uint8_t* h_pk[2]{};  // pinned packets of a collected batch, per packet set
    // Written at the end of each batch by kernels on the coder stream, so
    // that collecting a batch needs no GPU work but one D2H copy (a small
    // copy or kernel issued then would queue behind the next batch's frames
    // or kernels): mapped pinned packet sizes per packet set, the
    // slice-budget status per status set, the packets back to back in HBM
    int64_t* h_sizes[2]{};
    int64_t* hd_sizes[2]{};  // their device-side address
    int* h_status = nullptr;  // [2][4]
    int* hd_status = nullptr;
    int64_t h_pk_cap[2]{};
    // 10-bit samples in 16-bit words cross PCIe packed three to a 32-bit
    // word (pack10_rows), into a packed area per frame set that
    // ffv1_unpack10 expands into the frame slots; rawf: frames staged as is
    bool pack10 = false;
    uint8_t* d_packed[3]{};
    int64_t packed_frame_bytes = 0;
    int64_t poff[kMaxPlanes]{};
    int pw[kMaxPlanes]{}, prow[kMaxPlanes]{};  // samples per row, packed bytes per row
    std::vector<uint8_t> rawf[3];
    uint8_t* d_compact[2]{};  // the same, back to back in HBM (one D2H copy)
    int64_t d_compact_cap[2]{};
    // FFV1HIP_DEBUG=hostdbg (measurement hook): where ffv1hip_encode's host time
    // goes, seconds: waiting for a staging slot, copying into slots, issuing
    // their DMA, waiting for the copy-out thread, settling a batch, and in
    // the copy-out: packets over PCIe, into the caller's buffer
    bool dbg = false;
    double t_slot = 0, t_copy = 0, t_dma = 0, t_join = 0, t_settle = 0, t_d2h = 0, t_out = 0;
    double t_sizes = 0, t_compact = 0, t_dcopy = 0;  // inside the D2H (hostdbg)
  } pipe;
  uint8_t* d_frames2 = nullptr;
  uint8_t* d_frames3 = nullptr;
  // encode2 with the pipe: the set being filled and the launched batches
  // whose packets are not handed out yet (batch id, pts)
  int q_set = 0;
  // caller-pinned host ranges (ffv1hip_host_register): begin -> {bytes,
  // pinned here}; frames inside one go to HBM straight from the caller
  struct HostRange {
    int64_t bytes;
    bool owned;
  };
  std::map<uintptr_t, HostRange> host_ranges;
  bool direct_pending = false;  // a direct copy was queued on the transfer stream
  hipEvent_t direct_ev = nullptr;
  int64_t last_out = -1;  // the packet the last encode2 call handed out (ready index), -1: none
  struct Launched {
    int64_t b;
    std::vector<int64_t> pts;
  };
  std::deque<Launched> launched;
};

extern "C" {

const char* ffv1hip_last_error(void) { return g_err; }
int ffv1hip_abi_version(void) { return FFV1HIP_ABI_VERSION; }

int64_t ffv1hip_debug_counter(const ffv1hip_ctx* c, const char* name) {
  if (!c || !name) return -1;
  if (!std::strcmp(name, "guard_skips")) return c->guard_skips;
  if (!std::strcmp(name, "guard_reruns")) return c->guard_reruns;
  return -1;
}

int ffv1hip_debug_checks(void) { return kBoundsCheck ? 1 : 0; }

int ffv1hip_configure(ffv1hip_params* out, const ffv1hip_options* o) {
  if (!out || !o || !o->pix_fmt || o->width <= 0 || o->height <= 0)
    return set_err(-22, "invalid arguments");
  // rgb: 1 AV_PIX_FMT_0RGB32 (bgr0 bytes) / RGB32 (bgra bytes), 2 GBRP9..14
  // (ffv1enc.c:780-814); planes = the format's components (2 and 4: alpha)
  struct Fmt { const char* name; int planes, hs, vs, depth, rgb; };
  static const Fmt fmts[] = {
      {"yuv420p", 3, 1, 1, 8, 0},    {"yuv422p", 3, 1, 0, 8, 0},    {"yuv444p", 3, 0, 0, 8, 0},
      {"yuv440p", 3, 0, 1, 8, 0},    {"yuv411p", 3, 2, 0, 8, 0},    {"yuv410p", 3, 2, 2, 8, 0},
      {"gray", 1, 0, 0, 8, 0},       {"yuv420p9", 3, 1, 1, 9, 0},   {"yuv422p9", 3, 1, 0, 9, 0},
      {"yuv444p9", 3, 0, 0, 9, 0},   {"yuv420p10", 3, 1, 1, 10, 0}, {"yuv422p10", 3, 1, 0, 10, 0},
      {"yuv444p10", 3, 0, 0, 10, 0}, {"yuv420p16", 3, 1, 1, 16, 0}, {"yuv422p16", 3, 1, 0, 16, 0},
      {"yuv444p16", 3, 0, 0, 16, 0}, {"gray16", 1, 0, 0, 16, 0},    {"bgr0", 3, 0, 0, 8, 1},
      {"0rgb32", 3, 0, 0, 8, 1},     {"gbrp9", 3, 0, 0, 9, 2},      {"gbrp10", 3, 0, 0, 10, 2},
      {"gbrp12", 3, 0, 0, 12, 2},    {"gbrp14", 3, 0, 0, 14, 2},
      // with alpha (ffv1enc.c:725-786)
      {"yuva420p", 4, 1, 1, 8, 0},   {"yuva422p", 4, 1, 0, 8, 0},   {"yuva444p", 4, 0, 0, 8, 0},
      {"ya8", 2, 0, 0, 8, 0},        {"yuva420p9", 4, 1, 1, 9, 0},  {"yuva422p9", 4, 1, 0, 9, 0},
      {"yuva444p9", 4, 0, 0, 9, 0},  {"yuva420p10", 4, 1, 1, 10, 0}, {"yuva422p10", 4, 1, 0, 10, 0},
      {"yuva444p10", 4, 0, 0, 10, 0}, {"yuva420p16", 4, 1, 1, 16, 0}, {"yuva422p16", 4, 1, 0, 16, 0},
      {"yuva444p16", 4, 0, 0, 16, 0}, {"bgra", 4, 0, 0, 8, 1},      {"rgb32", 4, 0, 0, 8, 1},
  };
  const Fmt* f = nullptr;
  for (const Fmt& c : fmts)
    if (!std::strcmp(c.name, o->pix_fmt)) f = &c;
  if (!f) return set_err(-38, "pix_fmt %s not supported", o->pix_fmt);

  ffv1hip_params p{};
  p.width = o->width;
  p.height = o->height;
  p.gop_size = o->gop_size;
  p.sar_num = 0;
  p.sar_den = 1;
  // version (ffv1enc.c:678-706)
  int version = 0;
  if (o->pass || o->slices > 1) version = 2;  // AV_CODEC_FLAG_PASS1 | PASS2 (ffv1enc.c:680-682)
  if (o->slices == 0 && o->level < 0 && int64_t(o->width) * o->height > 720 * 576) version = 2;
  if (o->level <= 0 && version == 2) version = 3;
  if (o->level >= 0 && o->level <= 4) {
    if (o->level < version) return set_err(-22, "version %d needed, level %d requested", version, o->level);
    version = o->level;
  }
  p.ec = o->slicecrc < 0 ? (version >= 3) : o->slicecrc;
  if ((version == 2 || version > 3) && !o->experimental)
    return set_err(FFV1HIP_AVERROR_INVALIDDATA, "version %d is experimental in the reference", version);
  // version 2's extradata has no ec field (ffv1enc.c:593-598): its slice
  // CRCs would be unreadable by the reference decoder
  if (version == 2 && p.ec) return set_err(-38, "version 2 with slice CRCs (no ec field in its extradata)");
  // coder (ffv1enc.c:708-718)
  int ac = 0;
  if (o->coder != -1) ac = o->coder > 0 ? 2 : 0;
  if (o->coder == -2) ac = 1;
  // sample format (ffv1enc.c:720-820)
  int bits = 0, packed = 0;
  if (f->rgb == 1) {
    bits = o->bits_per_raw_sample ? o->bits_per_raw_sample : 8;
    if (bits != 8) return set_err(-38, "bgr0 with %d bits", bits);
  } else if (f->rgb == 2) {  // GBRPn: bits from the format, raw u16 samples
    bits = o->bits_per_raw_sample ? o->bits_per_raw_sample : f->depth;
    packed = 1;
    if (ac == 0) ac = 2;
    version = std::max(version, 1);
  } else if (f->depth > 8) {
    if (f->depth == 9 && !o->bits_per_raw_sample) bits = 9;
    if (f->depth <= 10) {
      packed = 1;
      if (!o->bits_per_raw_sample && !bits) bits = 10;
    }
    if (!o->bits_per_raw_sample && !bits) bits = 16;
    else if (!bits) bits = o->bits_per_raw_sample;
    if (bits <= 8) return set_err(FFV1HIP_AVERROR_INVALIDDATA, "bits_per_raw_sample invalid");
    if (ac == 0) ac = 2;  // >8 bit forces the range coder
    version = std::max(version, 1);
  }
  if (!bits) bits = 8;
  if (o->context < 0 || o->context > 1) return set_err(-22, "context model %d", o->context);
  // chroma_planes = nb_components >= 3, transparency = 4 or 2 components
  // (ffv1enc.c:772-774, 782)
  p.chroma_planes = f->planes >= 3;
  p.chroma_h_shift = f->planes >= 3 ? f->hs : 0;
  p.chroma_v_shift = f->planes >= 3 ? f->vs : 0;
  p.transparency = f->planes == 4 || f->planes == 2;
  p.bits_per_raw_sample = bits;
  p.packed_at_lsb = packed;
  p.sample_bytes = f->rgb == 1 ? 4 : f->depth > 8 ? 2 : 1;
  p.colorspace = f->rgb != 0;
  p.version = version;
  p.ac = ac;
  p.context_model = o->context;
  p.num_h_slices = p.num_v_slices = 1;
  // v4 runs choose_rct_params on every slice (ffv1enc.c:1163-1164): it reads
  // plane 0 as 32-bit B, G, R words at 8 bit, planes 0-2 as u16 at the luma
  // position above; inside the frame for RGB and >8-bit 4:4:4 YCbCr only
  if (version > 3 && !p.colorspace &&
      !(p.chroma_planes && !p.chroma_h_shift && !p.chroma_v_shift && p.sample_bytes == 2))
    return set_err(-38, "version 4 with %s: the reference reads outside the frame (choose_rct_params)", o->pix_fmt);
  // slice grid (ffv1enc.c:988-1000); allow_large_grid extends it to the
  // decoder's MAX_SLICES=256 (ffv1.h:77) for 8K.
  if (version > 1) {
    const int max_v = o->allow_large_grid ? 16 : 8;
    const int max_slices = o->allow_large_grid ? 256 : 64;
    int nv = (o->width > 352 || o->height > 288 || !o->slices) ? 2 : 1;
    bool ok = false;
    for (; nv <= max_v && !ok; nv++)
      for (int nh = nv; nh < 2 * nv && !ok; nh++)
        if ((o->slices == nh * nv && o->slices <= max_slices) || !o->slices) {
          p.num_h_slices = nh;
          p.num_v_slices = nv;
          ok = true;
        }
    if (!ok) return set_err(-38, "unsupported number of slices %d", o->slices);
  }
  *out = p;
  return 0;
}

// YA8: gray with alpha, Y and A bytes interleaved in one plane
// (ffv1enc.c:1199-1201)
static bool is_ya8(const ffv1hip_params& p) { return p.transparency && !p.chroma_planes && !p.colorspace; }

// Input planes of a frame (the caller's plane arrays): Y, Cb, Cr (+ A); one
// for gray, YA8, bgr0 and RGB32.
static int input_planes(const ffv1hip_params& p) {
  if (p.colorspace) return p.sample_bytes == 4 ? 1 : 3;
  return p.chroma_planes ? 3 + (p.transparency != 0) : 1;
}

static int build_extradata(ffv1hip_ctx* c) {
  const ffv1hip_params& p = c->P;
  c->extradata.clear();
  if (p.version < 2) return 0;
  HostRac r(&c->dflt);
  uint8_t st[32];
  std::memset(st, 128, 32);
  r.symbol(st, p.version, false);
  if (p.version > 2) r.symbol(st, p.version == 3 ? 4 : 2, false);
  r.symbol(st, p.ac, false);
  if (p.ac == 2)
    for (int i = 1; i < 256; i++) r.symbol(st, c->frame.to1[i] - c->dflt.to1[i], true);
  r.symbol(st, p.colorspace, false);
  r.symbol(st, p.bits_per_raw_sample, false);
  r.put(st, p.chroma_planes);
  r.symbol(st, p.chroma_h_shift, false);
  r.symbol(st, p.chroma_v_shift, false);
  r.put(st, p.transparency);
  r.symbol(st, p.num_h_slices - 1, false);
  r.symbol(st, p.num_v_slices - 1, false);
  r.symbol(st, 2, false);  // quant_table_count
  for (int set = 0; set < 2; set++) {
    int16_t qt[5][256];
    quant_set(qt, set, p.bits_per_raw_sample);
    for (int t = 0; t < 5; t++) {
      uint8_t qs[32];
      std::memset(qs, 128, 32);
      int last = 0, i;
      for (i = 1; i < 128; i++)
        if (qt[t][i] != qt[t][i - 1]) { r.symbol(qs, i - last - 1, false); last = i; }
      r.symbol(qs, i - last - 1, false);
    }
  }
  uint8_t st2[32][32];
  std::memset(st2, 128, sizeof(st2));
  for (int set = 0; set < 2; set++) {  // initial states (ffv1enc.c:591-607)
    const std::vector<uint8_t>& is = c->init_states[set];
    const bool any = std::any_of(is.begin(), is.end(), [](uint8_t v) { return v != 128; });
    r.put(st, any);
    if (!any) continue;
    for (size_t i = 0; i < is.size(); i++) {
      const int pred = i >= 32 ? is[i - 32] : 128;
      r.symbol(st2[i & 31], int8_t(is[i] - pred), true);
    }
  }
  if (p.version > 2) {
    r.symbol(st, p.ec, false);
    r.symbol(st, p.gop_size < 2, false);
  }
  r.finish();
  c->extradata = r.out;
  uint32_t crc = crc32_msb(c->extradata.data(), c->extradata.size());
  for (int k = 3; k >= 0; k--) c->extradata.push_back(uint8_t(crc >> (8 * k)));
  return 0;
}

// Decision-stream mode: a slice slot holds the values of low at the
// stream's shifts as u32 (about one per output byte) with a segment's worth
// of slack, which ffv1_sink then overwrites with the bytes.
static int64_t slice_stride_frames(int64_t slice_cap) { return 4 * (slice_cap + kSeg + 64); }

// Header programs: per (key, slice), the decisions coded before the planes.
static void build_ops(ffv1hip_ctx* c) {
  const ffv1hip_params& p = c->P;
  c->ops.assign(size_t(2) * c->nslices * kMaxOps, Op{0, 0, 0, 0});
  c->nops.assign(size_t(2) * c->nslices, 0);
  // the sets a v3 stream uses first: its coder then keeps only two per lane
  enum { kSetKey = 0, kSetSlice = 1, kSetHdr = 2, kSetQ0 = 3 };
  for (int key = 0; key < 2; key++)
    for (int s = 0; s < c->nslices; s++) {
      OpList L;
      if (s == 0) {
        L.bit(kSetKey, 0, key);  // key bit, state 128, default table
        if (key && p.version < 2) {  // write_header (ffv1enc.c:506-522)
          L.sym(kSetHdr, 0, p.version, false);
          L.sym(kSetHdr, 0, p.ac, false);
          if (p.ac == 2)
            for (int i = 1; i < 256; i++) L.sym(kSetHdr, 0, c->frame.to1[i] - c->dflt.to1[i], true);
          L.sym(kSetHdr, 0, p.colorspace, false);
          if (p.version > 0) L.sym(kSetHdr, 0, p.bits_per_raw_sample, false);
          L.bit(kSetHdr, 0, p.chroma_planes);
          L.sym(kSetHdr, 0, p.chroma_h_shift, false);
          L.sym(kSetHdr, 0, p.chroma_v_shift, false);
          L.bit(kSetHdr, 0, p.transparency);
          for (int t = 0; t < 5; t++) {
            int last = 0, i;
            for (i = 1; i < 128; i++)
              if (c->qt[t][i] != c->qt[t][i - 1]) { L.sym(kSetQ0 + t, 0, i - last - 1, false); last = i; }
            L.sym(kSetQ0 + t, 0, i - last - 1, false);
          }
        } else if (key && p.version == 2) {  // write_header (ffv1enc.c:523-541): the grid in band
          const int nh = p.num_h_slices, nv = p.num_v_slices;
          L.sym(kSetHdr, 0, c->nslices, false);
          for (int j = 0; j < c->nslices; j++) {
            const int jx = j % nh, jy = j / nh;
            const int x0 = int(int64_t(p.width) * jx / nh), x1 = int(int64_t(p.width) * (jx + 1) / nh);
            const int y0 = int(int64_t(p.height) * jy / nv), y1 = int(int64_t(p.height) * (jy + 1) / nv);
            L.sym(kSetHdr, 0, int(int64_t(x0 + 1) * nh / p.width), false);
            L.sym(kSetHdr, 0, int(int64_t(y0 + 1) * nv / p.height), false);
            L.sym(kSetHdr, 0, int(int64_t(x1 - x0 + 1) * nh / p.width) - 1, false);
            L.sym(kSetHdr, 0, int(int64_t(y1 - y0 + 1) * nv / p.height) - 1, false);
            for (int k = 0; k < c->pcount; k++) L.sym(kSetHdr, 0, p.context_model, false);
          }
        }
      }
      if (p.version > 2) {  // encode_slice_header (ffv1enc.c:1031-1051)
        const int nh = p.num_h_slices, nv = p.num_v_slices;
        const int sx = s % nh, sy = s / nh;
        const int x0 = int(int64_t(p.width) * sx / nh), x1 = int(int64_t(p.width) * (sx + 1) / nh);
        const int y0 = int(int64_t(p.height) * sy / nv), y1 = int(int64_t(p.height) * (sy + 1) / nv);
        L.sym(kSetSlice, 1, int(int64_t(x0 + 1) * nh / p.width), false);
        L.sym(kSetSlice, 1, int(int64_t(y0 + 1) * nv / p.height), false);
        L.sym(kSetSlice, 1, int(int64_t(x1 - x0 + 1) * nh / p.width) - 1, false);
        L.sym(kSetSlice, 1, int(int64_t(y1 - y0 + 1) * nv / p.height) - 1, false);
        for (int j = 0; j < c->pcount; j++) L.sym(kSetSlice, 1, p.context_model, false);
        L.sym(kSetSlice, 1, 3, false);  // progressive
        L.sym(kSetSlice, 1, p.sar_num, false);
        L.sym(kSetSlice, 1, p.sar_den, false);
        if (p.version > 3) {  // ffv1enc.c:1052-1061: slice_coding_mode (0, or 1 for PCM), the RCT coefficients
          L.ops.push_back(Op{int16_t(kOpBitMode), uint8_t(kSetSlice), 1, 0});
          L.ops.push_back(Op{int16_t(kOpSymMode), uint8_t(kSetSlice), 1, 0});
          L.ops.push_back(Op{int16_t(kOpSymRct), uint8_t(kSetSlice), 1, 0});
          L.ops.push_back(Op{int16_t(kOpSymRct), uint8_t(kSetSlice), 1, 1});
        }
      }
      const size_t sel = size_t(key) * c->nslices + s;
      c->nops[sel] = int(L.ops.size());
      std::memcpy(&c->ops[sel * kMaxOps], L.ops.data(), L.ops.size() * sizeof(Op));
    }
}

// The header decisions of each (key, slice) stream (the op programs above)
// do not depend on the pixels, so the decision-stream coder starts every
// stream after them: low, range and the values of low at their shifts
// (renorm_encoder's input, rangecoder.h:52-75), coded here once.
static void build_hdr(ffv1hip_ctx* c) {
  c->hdr.assign(size_t(2) * c->nslices, HdrState{0, 0xFF00, 0, 0});
  c->hdr_digits.clear();
  for (int key = 0; key < 2; key++)
    for (int s = 0; s < c->nslices; s++) {
      const size_t sel = size_t(key) * c->nslices + s;
      uint8_t os[kOpSets][32];
      std::memset(os, 128, sizeof(os));
      int low = 0, range = 0xFF00;
      const int off = int(c->hdr_digits.size());
      auto put = [&](uint8_t* st, int bit, const Tables& t) {
        const int r1 = (range * *st) >> 8;
        if (bit) {
          low += range - r1;
          range = r1;
          *st = t.to1[*st];
        } else {
          range -= r1;
          *st = t.to0[*st];
        }
        while (range < 0x100) {
          c->hdr_digits.push_back(uint32_t(low));
          low = (low & 0xFF) << 8;
          range <<= 8;
        }
      };
      for (int q = 0; q < c->nops[sel]; q++) {
        const Op& op = c->ops[sel * kMaxOps + q];
        const Tables& t = op.tab ? c->frame : c->dflt;
        uint8_t* st = os[op.set];
        if (op.kind == kOpBit) {
          put(st, op.value, t);
          continue;
        }
        const int v = op.value;
        if (!v) {
          put(st, 1, t);
          continue;
        }
        const unsigned a = v < 0 ? 0u - unsigned(v) : unsigned(v);
        const int e = 31 - __builtin_clz(a);
        put(st, 0, t);
        for (int i = 0; i < e; i++) put(st + 1 + std::min(i, 9), 1, t);
        put(st + 1 + std::min(e, 9), 0, t);
        for (int i = e - 1; i >= 0; i--) put(st + 22 + std::min(i, 9), (a >> i) & 1, t);
        if (op.kind == kOpSymS) put(st + 11 + std::min(e, 10), v < 0, t);
      }
      c->hdr[sel] = HdrState{low, range, int(c->hdr_digits.size()) - off, off};
    }
}

static int upload_hdr(ffv1hip_ctx* c) {
  if (!c->frames_mode) return 0;
  // build_hdr codes every op with its host value: a device-valued op (v4's
  // per-slice RCT coefficients) would come out wrong, so the frame-parallel
  // mode must never see one (it admits version <= 3 only, ffv1hip_create)
  for (size_t sel = 0; sel < c->nops.size(); sel++)
    for (int q = 0; q < c->nops[sel]; q++)
      if (c->ops[sel * kMaxOps + q].kind > kOpBit)
        return set_err(-5, "internal: a device-valued header op in the frame-parallel mode");
  if (c->d_hdr) HIP_TRY(hipFree(c->d_hdr));
  if (c->d_hdr_digits) HIP_TRY(hipFree(c->d_hdr_digits));
  c->d_hdr = nullptr;
  c->d_hdr_digits = nullptr;
  HIP_TRY(hipMalloc(&c->d_hdr, sizeof(HdrState) * c->hdr.size()));
  HIP_TRY(hipMemcpy(c->d_hdr, c->hdr.data(), sizeof(HdrState) * c->hdr.size(), hipMemcpyHostToDevice));
  HIP_TRY(hipMalloc(&c->d_hdr_digits, sizeof(uint32_t) * (c->hdr_digits.size() + 1)));
  if (!c->hdr_digits.empty())
    HIP_TRY(hipMemcpy(c->d_hdr_digits, c->hdr_digits.data(), sizeof(uint32_t) * c->hdr_digits.size(),
                      hipMemcpyHostToDevice));
  return 0;
}

static void pipe_close(ffv1hip_ctx* c);

// walktrace: per traced batch and launch part, when its waves
// started (spread from the batch's first), how long they ran, when the
// last ended (ms).
static void dump_walk_trace(ffv1hip_ctx* c) {
  if (!c->d_trace || !c->trace_n) return;
  std::vector<uint64_t> t(size_t(kTraceWords) * c->trace_items * c->trace_n);
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpy(t.data(), c->d_trace, t.size() * 8, hipMemcpyDeviceToHost) != hipSuccess)
    return;
  // walktrace=<path>: every wave's start, end (s_memrealtime), HW_ID and XCC_ID
  const std::string path = c->knobs.str("walktrace");
  if (!path.empty()) {
    if (FILE* fp = std::fopen(path.c_str(), "w")) {
      std::fprintf(fp, "batch,item,start,end,hw_id,xcc_id,loop_cycles,steps,wave_cycles\n");
      for (int b = 0; b < c->trace_n; b++)
        for (int i = 0; i < c->trace_items; i++) {
          const uint64_t* w = t.data() + size_t(kTraceWords) * (size_t(c->trace_items) * b + i);
          if (w[0])
            std::fprintf(fp, "%d,%d,%llu,%llu,%llu,%llu,%llu,%llu,%llu\n", b, i, (unsigned long long)w[0],
                         (unsigned long long)w[1], (unsigned long long)w[2], (unsigned long long)w[3],
                         (unsigned long long)w[4], (unsigned long long)w[5], (unsigned long long)w[6]);
        }
      std::fclose(fp);
    }
  }
  uint64_t prev_end = 0;
  for (int b = 0; b < c->trace_n; b++) {
    const uint64_t* w = t.data() + size_t(kTraceWords) * c->trace_items * b;
    int n = 0;
    while (n < c->trace_items && w[kTraceWords * n]) n++;
    if (!n) continue;
    uint64_t t0 = ~0ull;
    for (int i = 0; i < n; i++) t0 = std::min(t0, w[kTraceWords * i]);
    const int first = c->trace_first[b] ? c->trace_first[b] : n;
    for (int part = 0; part < 2; part++) {
      const int lo = part ? first : 0, hi = part ? n : first;
      if (lo >= hi) continue;
      uint64_t s0 = ~0ull, s1 = 0, e1 = 0;
      double dur = 0, dmax = 0;
      for (int i = lo; i < hi; i++) {
        s0 = std::min(s0, w[kTraceWords * i]);
        s1 = std::max(s1, w[kTraceWords * i]);
        e1 = std::max(e1, w[kTraceWords * i + 1]);
        const double d = double(w[kTraceWords * i + 1] - w[kTraceWords * i]) / 1e5;
        dur += d;
        dmax = std::max(dmax, d);
      }
      std::fprintf(stderr, "walktrace batch %d part %c: %d waves, start %.2f..%.2f ms, run mean %.2f max %.2f ms, "
                           "end %.2f ms%s\n", b, part ? 'B' : 'A', hi - lo, double(s0 - t0) / 1e5,
                   double(s1 - t0) / 1e5, dur / (hi - lo), dmax, double(e1 - t0) / 1e5,
                   part == 0 && prev_end ? "" : "");
    }
    if (prev_end)
      std::fprintf(stderr, "walktrace batch %d: starts %.2f ms after batch %d's last wave ended\n", b,
                   (double(t0) - double(prev_end)) / 1e5, b - 1);
    prev_end = 0;
    for (int i = 0; i < n; i++) prev_end = std::max(prev_end, w[kTraceWords * i + 1]);
  }
}

static void free_device(ffv1hip_ctx* c) {
  dump_walk_trace(c);
  if (c->d_trace) (void)hipFree(c->d_trace);
  pipe_close(c);
  void* ptrs[] = {c->d_frames, c->d_qt, c->d_qt_walk, c->d_tabs, c->d_ops, c->d_nops, c->d_segs, c->d_keys,
                  c->d_slice_out, c->d_slice_bytes, c->d_packets, c->d_packet_size, c->d_persist[0],
                  c->d_persist[1], c->d_tables, c->d_sym, c->d_keys2, c->d_cbits, c->d_dcount, c->d_dbase, c->d_dtotal, c->d_pre[0],
                  c->d_pre[1], c->d_bits[0], c->d_bits[1], c->d_scratch, c->d_hdr, c->d_hdr_digits, c->d_geom, c->d_slot_frames, c->d_status,
                  c->d_rec2, c->d_cbits2, c->d_ident, c->d_segs_info, c->d_seg_totals, c->d_wmap, c->d_ck,
                  c->d_segrec, c->d_rct, c->d_bounds, c->d_rstate};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (c->h_dtotal) (void)hipHostFree(c->h_dtotal);
  if (c->h_tot_map) (void)hipHostFree(c->h_tot_map);
  for (hipEvent_t& e : c->ev)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t& e : c->kev)
    if (e) (void)hipEventDestroy(e);
  for (void* q : {(void*)c->d_rcstat, (void*)c->d_rcstat_bak, (void*)c->d_init})
    if (q) (void)hipFree(q);
  if (c->dep_ev) (void)hipEventDestroy(c->dep_ev);
  if (c->done_ev) (void)hipEventDestroy(c->done_ev);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->code_stream) (void)hipStreamDestroy(c->code_stream);
  if (c->bits_stream) (void)hipStreamDestroy(c->bits_stream);
  for (hipEvent_t& e : c->walked)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t& e : c->laid)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t& e : c->bitsed)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t& e : c->coded)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t& e : c->pre_read)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t& e : c->coded3)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t& e : c->entry)
    if (e) (void)hipEventDestroy(e);
  if (c->walk_a) (void)hipEventDestroy(c->walk_a);
  if (c->walk_go) (void)hipEventDestroy(c->walk_go);
  for (hipEvent_t& e : c->hist_done)
    if (e) (void)hipEventDestroy(e);
}

// Decision-stream buffers of set k for `need` decisions.  The set's previous
// user (the coder of batch k-2) must be done: the caller waits on coded[k].
static int grow_decisions(ffv1hip_ctx* c, int k, int64_t need) {
  if (need <= c->dcap[k]) return 0;
  if (c->d_pre[k]) HIP_TRY(hipFree(c->d_pre[k]));
  if (c->d_bits[k]) HIP_TRY(hipFree(c->d_bits[k]));
  c->d_pre[k] = nullptr;
  c->d_bits[k] = nullptr;
  c->dcap[k] = 0;
  const int64_t cap = (need + 4095) & ~int64_t(4095);
  HIP_TRY(hipMalloc(&c->d_pre[k], size_t(cap)));
  HIP_TRY(hipMalloc(&c->d_bits[k], size_t(cap / 8)));
  c->dcap[k] = cap;
  return 0;
}

// Decision-stream capacity of one set for a batch of nb frames: the worst
// case when it is small, else ~12 per symbol (real content codes ~3; a batch
// that needs more grows the set).
static int64_t decision_cap(const ffv1hip_ctx* c, int64_t nb) {
  const int64_t align = nb * c->nslices * kStreamSlack;
  const int64_t worst = nb * c->frame_samples * c->wmax + align;
  const int64_t guess = nb * c->frame_samples * 12 + align;
  const int64_t cap = worst <= (int64_t(1) << 31) ? worst : std::min(worst, guess);
  return (cap + 4095) & ~int64_t(4095);
}

// HBM the context's buffers take for a batch of nb frames (the second walk
// records set, allocated only with room to spare, and the host-frame path's
// frame slots, allocated on its first use, not counted).
// The slice byte budget a large batch can go down to (alloc_rec2): a
// quarter, or 1/q with budget=q; else the budget as it is.
static int64_t low_slice_cap(const ffv1hip_ctx* c) {
  const int64_t q = c->knobs.get("budget", 4);
  if (!c->lazy_sets || q <= 1 || c->knobs.has("slice_cap")) return c->slice_cap;
  return std::min(c->slice_cap, ((c->slice_cap - 4096) / q + 4096 + 255) & ~int64_t(255));
}

static int64_t device_bytes(const ffv1hip_ctx* c, int64_t nb) {
  // (a large batch counted at the budget it can go down to)
  const int64_t cap = low_slice_cap(c);
  const int64_t stride = c->frames_mode ? slice_stride_frames(cap) : cap;
  int64_t b = nb * (stride * c->nslices + (((cap + 16) * c->nslices + 255) & ~int64_t(255)));
  b += 2 * int64_t(c->pcount) * c->contexts * 32 * c->nslices;  // the P-frame carry
  if (c->frames_mode) {
    b += nb * (8 * c->frame_samples + 4 * int64_t(c->cwords) * c->frame_chunks);  // walk records, chunk bits
    const int64_t dcap = decision_cap(c, nb);
    b += 2 * (dcap + dcap / 8);                                                      // two decision sets
    int64_t segs = 0, groups = 0;
    for (const SliceGeom& g : c->geom) {
      const int64_t l = int64_t(g.pw[0]) * g.ph[0] * c->wmax;
      const int64_t ch = (int64_t(g.pw[1]) * g.ph[1] + int64_t(g.pw[2]) * g.ph[2]) * c->wmax;
      const int64_t n = std::max<int64_t>(1, (l + kSeg - 1) / kSeg + (ch + kSeg - 1) / kSeg);
      segs += n;
      groups += (n + 63) / 64;
    }
    b += nb * (2 * 8 * segs + 3 * 4 * groups);  // checkpoints, segment records, group maps
  } else {
    const int64_t slots = c->max_slots;
    b += slots * (4 * c->frame_samples + int64_t(c->pcount) * c->contexts * 32 * c->nslices);
  }
  return b;
}

// The second set of walk records and chunk bits, only with room to spare:
// set 1 before its first batch counts as large as set 0, and a later batch
// may still grow the sets by an eighth (plus 2 GB for the runtime).  Beyond
// that, ensure_decisions gives the second set back.
static int alloc_rec2(ffv1hip_ctx* c) {
  if (!c->rec2_pending) return 0;
  c->rec2_pending = false;
  const int nb = c->max_batch;
  const size_t rec_bytes = sizeof(uint2) * size_t(c->frame_samples) * nb;
  const size_t cb_bytes = sizeof(uint32_t) * c->cwords * size_t(c->frame_chunks) * nb;
  size_t free_b = 0, total_b = 0;
  HIP_TRY(hipMemGetInfo(&free_b, &total_b));
  const size_t d0 = size_t(c->dcap[0]), d1 = c->dcap[1] ? size_t(c->dcap[1]) : d0;
  const size_t unsized = c->dcap[1] ? 0 : d1 + d1 / 8;  // set 1, still to come
  const size_t margin = unsized + (d0 + d1) / 8 + (size_t(2) << 30);
  // no room, in the first batch (its coder has not run): the slice byte
  // budget goes down to a quarter and a slice over it encodes its batch
  // again with a budget sized from what it needed (budget=q: down to 1/q,
  // room or not)
  if ((free_b <= rec_bytes + cb_bytes + margin || c->knobs.has("budget")) && c->nsub == 0) {
    const int64_t cap = low_slice_cap(c);
    if (cap < c->slice_cap) {
      HIP_TRY(hipDeviceSynchronize());
      for (uint8_t** b : {&c->d_slice_out, &c->d_packets, &c->d_packets2}) {
        if (*b) HIP_TRY(hipFree(*b));
        *b = nullptr;
      }
      c->slice_cap = cap;
      c->slice_stride = slice_stride_frames(cap);
      c->packet_stride = ((cap + 16) * c->nslices + 255) & ~int64_t(255);
      const size_t pk_bytes = size_t(c->packet_stride) * nb;
      HIP_TRY(hipMalloc(&c->d_slice_out, size_t(c->slice_stride) * c->nslices * nb));
      HIP_TRY(hipMalloc(&c->d_packets, pk_bytes));
      if (c->two_pk) HIP_TRY(hipMalloc(&c->d_packets2, pk_bytes));
      HIP_TRY(hipMemGetInfo(&free_b, &total_b));
    }
  }
  if (free_b > rec_bytes + cb_bytes + margin) {
    if (hipMalloc(&c->d_rec2, rec_bytes) == hipSuccess && hipMalloc(&c->d_cbits2, cb_bytes) == hipSuccess) {
      c->two_rec = true;
    } else {
      (void)hipGetLastError();
      if (c->d_rec2) (void)hipFree(c->d_rec2);
      c->d_rec2 = nullptr;
    }
  }
  if (c->knobs.has("hostdbg"))
    std::fprintf(stderr, "hostdbg: decision sets %.2f / %.2f GB, %.2f GB free, second records set (%.2f GB + "
                         "margin %.2f GB): %s; slice budget %lld bytes\n", double(c->dcap[0]) / 1e9, double(c->dcap[1]) / 1e9,
                 double(free_b) / 1e9, double(rec_bytes + cb_bytes) / 1e9, double(margin) / 1e9,
                 c->two_rec ? "yes" : "no", (long long)c->slice_cap);
  return 0;
}

// Decision set fb for `need` decisions (a batch's, read back after its
// layout).  When HBM does not hold the larger set beside two records sets,
// the records set this batch does not use is given back (after every stream
// of the context has drained) and the context goes on with one set: the one
// holding this batch's records becomes set 0.  *rec / *cbits: this batch's.
static int ensure_decisions(ffv1hip_ctx* c, int fb, int64_t need, uint2** rec, uint32_t** cbits) {
  const int64_t want = need + need / 8;
  // rec2_drop=k (test hook): as if set fb = k did not fit beside two records sets
  const bool drop_hook = c->two_rec && c->knobs.has("rec2_drop") && c->knobs.get("rec2_drop", 0) == fb;
  if (!drop_hook) {
    if (grow_decisions(c, fb, want) == 0) {
      if (c->rec2_pending) return alloc_rec2(c);
      return 0;
    }
    (void)hipGetLastError();
    if (!c->two_rec) return -1;
  }
  if (c->knobs.has("hostdbg"))
    std::fprintf(stderr, "hostdbg: decision set %d to %.2f GB: the second records set goes\n", fb, double(want) / 1e9);
  // every stream of the context drained: nothing reads either records set
  HIP_TRY(hipStreamSynchronize(c->stream));
  HIP_TRY(hipStreamSynchronize(c->code_stream));
  HIP_TRY(hipStreamSynchronize(c->bits_stream));
  uint2* const set0 = reinterpret_cast<uint2*>(c->d_sym);
  if (*rec == c->d_rec2) {  // this batch's records are in set 1: keep those
    HIP_TRY(hipFree(set0));
    HIP_TRY(hipFree(c->d_cbits));
    c->d_sym = reinterpret_cast<uint32_t*>(c->d_rec2);
    c->d_cbits = c->d_cbits2;
  } else {
    HIP_TRY(hipFree(c->d_rec2));
    HIP_TRY(hipFree(c->d_cbits2));
  }
  c->d_rec2 = nullptr;
  c->d_cbits2 = nullptr;
  c->two_rec = false;
  *rec = reinterpret_cast<uint2*>(c->d_sym);
  *cbits = c->d_cbits;
  return grow_decisions(c, fb, want);
}

// A batch whose decision sets would be sized by decision_cap's guess (its
// worst case is over 2^31 decisions) and that does not fit with both records
// sets that way is sized from its content instead: decision sets, the
// second records set and the slice byte budget (dsets=eager|lazy
// overrides).  (One that fits allocates everything at create: none of it
// lands in the first batches' time.)
static int64_t device_bytes(const ffv1hip_ctx* c, int64_t nb);
static bool lazy_sizing(const ffv1hip_ctx* c) {
  const int64_t nb = c->max_batch;
  const int64_t worst = nb * c->frame_samples * c->wmax + nb * c->nslices * kStreamSlack;
  const std::string ds = c->knobs.str("dsets");
  if (ds == "lazy") return true;
  const int64_t cap = decision_cap(c, nb);
  if (ds == "eager" || cap >= worst) return false;
  size_t free_b = 0, total_b = 0;
  if (hipSetDevice(c->device) != hipSuccess || hipMemGetInfo(&free_b, &total_b) != hipSuccess) return true;
  const int64_t rec2 = nb * (8 * c->frame_samples + 4 * int64_t(c->cwords) * c->frame_chunks);
  const int64_t eager = device_bytes(c, nb) + rec2 + cap / 2 + (int64_t(5) << 30);  // alloc_rec2's old margin
  return eager > int64_t(free_b);
}

static int alloc_device(ffv1hip_ctx* c) {
  HIP_TRY(hipSetDevice(c->device));
  const int nb = c->max_batch;
  {  // a batch that cannot fit is refused up front, with the largest one that can
    size_t free_b = 0, total_b = 0;
    HIP_TRY(hipMemGetInfo(&free_b, &total_b));
    const int64_t need = device_bytes(c, nb);
    const int64_t reserve = int64_t(1) << 30;  // streams, events, the runtime
    if (need + reserve > int64_t(free_b)) {
      int64_t fit = 0;
      for (int64_t lo = 1, hi = nb; lo <= hi;) {
        const int64_t mid = (lo + hi) / 2;
        if (device_bytes(c, mid) + reserve <= int64_t(free_b)) {
          fit = mid;
          lo = mid + 1;
        } else {
          hi = mid - 1;
        }
      }
      return set_err(-12, "a batch of %d frames needs %.1f GB of device memory, %.1f GB are free: "
                          "at most %lld frames per batch fit", nb, double(need) / 1e9, double(free_b) / 1e9,
                     (long long)fit);
    }
  }
  HIP_TRY(hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, c->device));
  HIP_TRY(hipDeviceGetAttribute(&c->lds_block, hipDeviceAttributeMaxSharedMemoryPerBlock, c->device));
  HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  for (hipEvent_t& e : c->hist_done) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIP_TRY(hipMalloc(&c->d_qt, sizeof(c->qt)));
  HIP_TRY(hipMemcpy(c->d_qt, c->qt, sizeof(c->qt), hipMemcpyHostToDevice));
  if (c->frames_mode && c->walk_rows != c->contexts) {
    int16_t qd[5][256] = {};
    const auto A = {5, 13, 27, 56};  // quant9_10bit's steps (quant_set, bits > 8)
    quant_table(qd[0], A, 1);
    quant_table(qd[1], A, 9);
    quant_table(qd[2], A, 81);
    HIP_TRY(hipMalloc(&c->d_qt_walk, sizeof(qd)));
    HIP_TRY(hipMemcpy(c->d_qt_walk, qd, sizeof(qd), hipMemcpyHostToDevice));
  }
  uint8_t tabs[1024];
  std::memcpy(tabs, c->dflt.to0, 256);
  std::memcpy(tabs + 256, c->dflt.to1, 256);
  std::memcpy(tabs + 512, c->frame.to0, 256);
  std::memcpy(tabs + 768, c->frame.to1, 256);
  HIP_TRY(hipMalloc(&c->d_tabs, 1024));
  HIP_TRY(hipMemcpy(c->d_tabs, tabs, 1024, hipMemcpyHostToDevice));
  HIP_TRY(hipMalloc(&c->d_ops, c->ops.size() * sizeof(Op)));
  HIP_TRY(hipMemcpy(c->d_ops, c->ops.data(), c->ops.size() * sizeof(Op), hipMemcpyHostToDevice));
  HIP_TRY(hipMalloc(&c->d_nops, c->nops.size() * sizeof(int)));
  HIP_TRY(hipMemcpy(c->d_nops, c->nops.data(), c->nops.size() * sizeof(int), hipMemcpyHostToDevice));
  HIP_TRY(hipMalloc(&c->d_segs, sizeof(Segment) * (nb + 1)));
  HIP_TRY(hipMalloc(&c->d_keys, nb));
  if (hipMalloc(&c->d_slice_out, size_t(c->slice_stride) * c->nslices * nb) != hipSuccess ||
      hipMalloc(&c->d_packets, size_t(c->packet_stride) * nb) != hipSuccess) {
    // a large batch: at the budget it can go down to (what device_bytes counted)
    (void)hipGetLastError();
    for (uint8_t** q : {&c->d_slice_out, &c->d_packets}) {
      if (*q) HIP_TRY(hipFree(*q));
      *q = nullptr;
    }
    const int64_t cap = low_slice_cap(c);
    if (cap >= c->slice_cap) return set_err(-12, "slice buffers for a %lld-byte budget", (long long)c->slice_cap);
    c->slice_cap = cap;
    c->slice_stride = slice_stride_frames(cap);
    c->packet_stride = ((cap + 16) * c->nslices + 255) & ~int64_t(255);
    HIP_TRY(hipMalloc(&c->d_slice_out, size_t(c->slice_stride) * c->nslices * nb));
    HIP_TRY(hipMalloc(&c->d_packets, size_t(c->packet_stride) * nb));
  }
  HIP_TRY(hipMalloc(&c->d_slice_bytes, sizeof(int64_t) * c->nslices * nb));
  HIP_TRY(hipMemset(c->d_slice_bytes, 0, sizeof(int64_t) * c->nslices * nb));
  HIP_TRY(hipMalloc(&c->d_packet_size, sizeof(int64_t) * nb));
  HIP_TRY(hipMemset(c->d_packet_size, 0, sizeof(int64_t) * nb));
  const size_t state_bytes = size_t(c->pcount) * c->contexts * 32;
  for (uint8_t*& pb : c->d_persist) {
    HIP_TRY(hipMalloc(&pb, state_bytes * c->nslices));
    HIP_TRY(hipMemset(pb, 128, state_bytes * c->nslices));
  }
  HIP_TRY(hipEventCreateWithFlags(&c->dep_ev, hipEventDisableTiming));
  HIP_TRY(hipEventCreateWithFlags(&c->done_ev, hipEventDisableTiming));
  for (hipEvent_t& e : c->entry) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  // the coder grid is padded to whole waves and idle lanes touch their own table
  if (c->frames_mode) {
    // double-buffered: the states walk of batch k+1 runs while batch k codes
    // the walk records and chunk bits: one set (the next batch's symbols run
    // after this batch's walk on the same stream, and wait for its bits)
    HIP_TRY(hipMalloc(&c->d_sym, sizeof(uint2) * size_t(c->frame_samples) * nb));
    HIP_TRY(hipMalloc(&c->d_keys2, 3 * size_t(nb)));
    HIP_TRY(hipMalloc(&c->d_cbits, sizeof(uint32_t) * c->cwords * size_t(c->frame_chunks) * nb));
    HIP_TRY(hipMalloc(&c->d_dcount, 3 * sizeof(int) * 3 * size_t(nb) * c->nslices));
    HIP_TRY(hipMalloc(&c->d_dbase, 3 * sizeof(int64_t) * size_t(nb) * c->nslices));
    HIP_TRY(hipMalloc(&c->d_dtotal, 3 * sizeof(int64_t)));
    HIP_TRY(hipHostMalloc(&c->h_dtotal, 3 * sizeof(int64_t), hipHostMallocDefault));
    HIP_TRY(hipHostMalloc(&c->h_tot_map, 3 * sizeof(int64_t), hipHostMallocMapped));
    HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->hd_tot_map), c->h_tot_map, 0));
    for (int k = 0; k < 3; k++) c->h_tot_map[k] = 0;
    for (hipEvent_t& e : c->coded3) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c->walk_a, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c->walk_go, hipEventDisableTiming));
    {
      std::vector<int> ident(nb);
      for (int i = 0; i < nb; i++) ident[i] = i;
      HIP_TRY(hipMalloc(&c->d_ident, sizeof(int) * size_t(nb)));
      HIP_TRY(hipMemcpy(c->d_ident, ident.data(), sizeof(int) * size_t(nb), hipMemcpyHostToDevice));
    }
    HIP_TRY(hipStreamCreateWithFlags(&c->code_stream, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&c->bits_stream, hipStreamNonBlocking));
    for (hipEvent_t& e : c->laid) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (hipEvent_t& e : c->bitsed) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (hipEvent_t& e : c->walked) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (hipEvent_t& e : c->coded) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (hipEvent_t& e : c->pre_read) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIP_TRY(hipMalloc(&c->d_scratch, 4096));
    if (kBoundsCheck) {
      HIP_TRY(hipMalloc(&c->d_bounds, sizeof(uint32_t)));
      HIP_TRY(hipMemset(c->d_bounds, 0, sizeof(uint32_t)));
    }
    // the coder's segments: at most wmax decisions per sample
    c->max_segs = 0;
    c->max_groups = 0;
    for (const SliceGeom& g : c->geom) {
      const int64_t l = int64_t(g.pw[0]) * g.ph[0] * c->wmax;
      const int64_t ch = (int64_t(g.pw[1]) * g.ph[1] + int64_t(g.pw[2]) * g.ph[2]) * c->wmax;
      const int64_t n = std::max<int64_t>(1, (l + kSeg - 1) / kSeg + (ch + kSeg - 1) / kSeg);
      c->max_segs += n * nb;
      c->max_groups += (n + 63) / 64 * nb;
    }
    HIP_TRY(hipMalloc(&c->d_segs_info, 3 * sizeof(StreamSegs) * size_t(nb) * c->nslices));
    HIP_TRY(hipMalloc(&c->d_seg_totals, 3 * 2 * sizeof(int)));
    HIP_TRY(hipMalloc(&c->d_wmap, 3 * sizeof(int) * size_t(c->max_groups)));
    HIP_TRY(hipMalloc(&c->d_ck, sizeof(uint2) * size_t(c->max_segs)));
    HIP_TRY(hipMalloc(&c->d_segrec, sizeof(uint2) * size_t(c->max_segs)));
    HIP_TRY(hipMalloc(&c->d_rstate, sizeof(int2) * size_t(nb) * c->nslices));
    if (upload_hdr(c) < 0) return -5;
    // Decision sets: a batch whose worst case is small gets it now; a large
    // one (the guess of decision_cap) is sized from what its first batches
    // need (ensure_decisions), and the second records set then takes the
    // room real content leaves (4:4:4 12-bit at 19 GOPs: ~3 decisions per
    // sample against the guess of 12, so both records sets fit beside them)
    const int64_t cap = decision_cap(c, nb);
    if (!c->lazy_sets)
      for (int k = 0; k < 2; k++)
        if (grow_decisions(c, k, cap) < 0) return -5;
    // the recsets=1 hook keeps one set
    c->rec2_pending = c->knobs.get("recsets", 2) != 1;
    if (!c->lazy_sets && alloc_rec2(c) < 0) return -5;
  } else {
    const size_t chains = (size_t(c->max_slots) * c->nslices + 63) & ~size_t(63);
    HIP_TRY(hipMalloc(&c->d_tables, state_bytes * (chains + 64)));  // + ffv1_code's 64 dummy tables
    c->table_dummy = int64_t(chains);
    HIP_TRY(hipMalloc(&c->d_sym, sizeof(uint32_t) * size_t(c->frame_samples) * c->max_slots));
  }
  HIP_TRY(hipMalloc(&c->d_geom, sizeof(SliceGeom) * c->nslices));
  HIP_TRY(hipMemcpy(c->d_geom, c->geom.data(), sizeof(SliceGeom) * c->nslices, hipMemcpyHostToDevice));
  HIP_TRY(hipMalloc(&c->d_slot_frames, sizeof(int) * size_t(c->max_slots) * (nb + 1)));
  if (c->P.version > 3) HIP_TRY(hipMalloc(&c->d_rct, sizeof(int2) * size_t(nb) * c->nslices));
  HIP_TRY(hipMalloc(&c->d_status, sizeof(int) * 8));
  HIP_TRY(hipMemset(c->d_status, 0, sizeof(int) * 8));
  return 0;
}

ffv1hip_ctx* ffv1hip_create(const ffv1hip_params* params, int device, int max_batch_frames, int* err) {
  auto fail = [&](int code) -> ffv1hip_ctx* {
    if (err) *err = code;
    return nullptr;
  };
  if (!params || max_batch_frames <= 0) return fail(set_err(-22, "invalid arguments"));
  const ffv1hip_params& p = *params;
  const bool fmt_ok = p.colorspace == 0   ? (p.sample_bytes == 1) == (p.bits_per_raw_sample == 8) && p.sample_bytes <= 2
                     : p.colorspace == 1 ? p.chroma_planes && !p.chroma_h_shift && !p.chroma_v_shift &&
                                               (p.sample_bytes == 4 ? p.bits_per_raw_sample == 8
                                                                    : p.sample_bytes == 2 && p.packed_at_lsb &&
                                                                          p.bits_per_raw_sample <= 14 && !p.transparency)
                                         : false;
  if (p.version > 4 || p.num_h_slices * p.num_v_slices > 256 || (p.version == 2 && p.ec) ||
      p.bits_per_raw_sample < 8 || p.bits_per_raw_sample > 16 || p.width <= 0 || p.height <= 0 || !fmt_ok)
    return fail(set_err(-38, "unsupported parameter set"));
  // version 2's keyframe header (2 + slices x (4 + planes) symbols) within
  // slice 0's header program: the reference grid (<= 64 slices) fits
  if (p.version == 2 && 2 + p.num_h_slices * p.num_v_slices * (6 + (p.transparency != 0)) > kMaxOps)
    return fail(set_err(-38, "version 2 with %d slices: its keyframe header exceeds %d header symbols",
                        p.num_h_slices * p.num_v_slices, kMaxOps));
  if (p.num_h_slices > p.width || p.num_v_slices > p.height)
    return fail(set_err(-22, "more slices than rows/columns"));
  ffv1hip_ctx* c = new ffv1hip_ctx();
  if (parse_knobs(&c->knobs) < 0) {
    delete c;
    return fail(-22);
  }
  c->P = p;
  c->device = device;
  c->max_batch = max_batch_frames;
  c->nslices = p.num_h_slices * p.num_v_slices;
  c->contexts = contexts_of(p.context_model);
  c->pcount = 2 + (p.transparency != 0);
  c->ncoded = p.colorspace ? 3 + (p.transparency != 0)
                           : p.chroma_planes ? 3 + (p.transparency != 0) : 1 + (p.transparency != 0);
  c->dflt = default_tables();
  c->frame = p.ac == 2 ? custom_tables(c->dflt) : c->dflt;
  quant_set(c->qt, p.context_model, p.bits_per_raw_sample);
  build_extradata(c);
  build_ops(c);
  build_hdr(c);
  // layout of a frame in the batch buffer (planar, tightly packed): Y, Cb,
  // Cr, A (YUVA); YA8 one plane of Y, A byte pairs; bgr0 / RGB32 one plane
  // of 4-byte pixels
  const bool ya8 = is_ya8(p);
  const int cw = p.chroma_planes ? -((-p.width) >> p.chroma_h_shift) : 0;
  const int ch = p.chroma_planes ? -((-p.height) >> p.chroma_v_shift) : 0;
  c->plane_bytes[0] = int64_t(p.width) * p.height * p.sample_bytes * (ya8 ? 2 : 1);
  c->plane_bytes[1] = c->plane_bytes[2] = p.sample_bytes == 4 ? 0 : int64_t(cw) * ch * p.sample_bytes;
  c->plane_bytes[3] = p.transparency && !p.colorspace && p.chroma_planes ? int64_t(p.width) * p.height * p.sample_bytes : 0;
  c->frame_bytes = (c->plane_bytes[0] + 2 * c->plane_bytes[1] + c->plane_bytes[3] + 255) & ~int64_t(255);
  // Per-slice geometry and symbol-stream layout (ffv1.c:117-145,
  // ffv1enc.c:1185-1196); each slice's stream is padded to 4 symbols.
  c->geom.resize(c->nslices);
  int64_t off = 0, max_nsym = 0;
  for (int s = 0; s < c->nslices; s++) {
    SliceGeom& g = c->geom[s];
    const int sx = s % p.num_h_slices, sy = s / p.num_h_slices;
    const int x0 = int(int64_t(p.width) * sx / p.num_h_slices);
    const int y0 = int(int64_t(p.height) * sy / p.num_v_slices);
    const int sw = int(int64_t(p.width) * (sx + 1) / p.num_h_slices) - x0;
    const int sh = int(int64_t(p.height) * (sy + 1) / p.num_v_slices) - y0;
    g.px[0] = x0; g.py[0] = y0; g.pw[0] = sw; g.ph[0] = sh;
    for (int k = 1; k < 3; k++) {
      g.pw[k] = p.chroma_planes ? -((-sw) >> p.chroma_h_shift) : 0;
      g.ph[k] = p.chroma_planes ? -((-sh) >> p.chroma_v_shift) : 0;
      g.px[k] = x0 >> p.chroma_h_shift;
      g.py[k] = y0 >> p.chroma_v_shift;
    }
    g.px[3] = g.py[3] = g.pw[3] = g.ph[3] = 0;
    if (p.transparency) {  // A at the luma rectangle: plane 3, or plane 1 of YA8
      const int k = ya8 ? 1 : 3;
      g.px[k] = x0; g.py[k] = y0; g.pw[k] = sw; g.ph[k] = sh;
    }
    int64_t n = 0;
    for (int k = 0; k < kMaxPlanes; k++) {
      g.plane_sym_off[k] = n;
      n += int64_t(g.pw[k]) * g.ph[k];
      g.chunk_off[k] = c->frame_chunks;
      c->frame_chunks += (int64_t(g.pw[k]) * g.ph[k] + 63) / 64;
    }
    g.nsym = n;
    g.sym_off = off;
    off += (n + 3) & ~int64_t(3);
    max_nsym = std::max(max_nsym, n);
  }
  c->frame_samples = off;
  // Slice byte budget: (bits + 4) / 8 bytes per coded sample (+4 KiB), above
  // what full-entropy noise codes to (~1.1 B per 8-bit, ~2.1 B per 16-bit
  // sample); a slice over it is encoded again with a budget sized from what
  // it needed (ffv1hip_fetch), as the reference codes any slice within its
  // w*h*140-byte packet (ffv1enc.c:1232).
  c->slice_cap = ((max_nsym * (std::max(8, p.bits_per_raw_sample) + 4) / 8 + 4096) + 255) & ~int64_t(255);
  // slice_cap (test hook): a small starting budget, to exercise the
  // re-encode with a larger one (ffv1hip_fetch)
  if (c->knobs.has("slice_cap"))
    c->slice_cap = (std::max<int64_t>(256, std::atoll(c->knobs.str("slice_cap").c_str())) + 255) & ~int64_t(255);
  c->packet_stride = ((c->slice_cap + 16) * c->nslices + 255) & ~int64_t(255);
  // frame slots (segments) per call: one per GOP touched by the batch
  c->max_slots = p.gop_size > 1 ? std::min(max_batch_frames, (max_batch_frames + p.gop_size - 2) / p.gop_size + 1)
                                : max_batch_frames;
  c->max_ops = 0;
  for (int v : c->nops) c->max_ops = std::max(c->max_ops, v);
  // Range coder with a table that fits the states walk's LDS: walk the
  // context states per GOP, recording every decision's state, then code all
  // (frame, slice) streams of a batch in parallel.  The coder=chain hook keeps
  // the chained per-GOP coder (a test hook: both must give equal bytes).
  {
    // dense rows above 8 bits with context model 0 (dense=0: the context
    // numbering, a test hook)
    const bool dense = p.context_model == 0 && p.bits_per_raw_sample > 8 && c->knobs.get("dense", 1) != 0;
    c->walk_rows = dense ? kDenseRows : c->contexts;
    // 8 bits, context model 0: rows of the 24 slots a symbol can use there
    // (compact=0: 32-byte rows, a test hook)
    c->walk_rowb = !dense && p.context_model == 0 && p.bits_per_raw_sample <= 8 && c->knobs.get("compact", 1) != 0
                       ? kCompactRowBytes
                       : 32;
    const int64_t lds = walk_lds_bytes(c->walk_rows, c->walk_rowb);
    // RGB interleaves the three planes' rows (encode_rgb_frame): chained
    // alpha (a third plane context) and v4 (per-frame slice header values):
    // the chained coders
    c->frames_mode = p.ac && !p.colorspace && !p.transparency && p.version <= 3 && lds <= kWalkLdsMax &&
                     c->knobs.str("coder") != "chain";
    c->wmax = 2 * (p.bits_per_raw_sample <= 8 ? 8 : p.bits_per_raw_sample) + 1;
    c->cwords = chunk_words(c->wmax);
    // a large batch, sized from what its content needs (lazy_sizing)
    c->lazy_sets = c->frames_mode && lazy_sizing(c);
    // the decision-stream coder writes a slice's digits (the values of low,
    // 4 bytes each) where ffv1_sink then writes its bytes
    c->slice_stride = c->frames_mode ? slice_stride_frames(c->slice_cap) : c->slice_cap;
  }
  int rc = alloc_device(c);
  if (rc < 0) {
    free_device(c);
    delete c;
    return fail(rc);
  }
  if (err) *err = 0;
  return c;
}

void ffv1hip_destroy(ffv1hip_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  free_device(c);  // (the transfer stream drained)
  for (const auto& r : c->host_ranges)
    if (r.second.owned) (void)hipHostUnregister(reinterpret_cast<void*>(r.first));
  if (c->direct_ev) (void)hipEventDestroy(c->direct_ev);
  if (c->xchg_ev) (void)hipEventDestroy(c->xchg_ev);
  delete c;
}

int ffv1hip_extradata(ffv1hip_ctx* c, uint8_t* buf, int cap) {
  if (!c) return set_err(-22, "null ctx");
  const int n = int(c->extradata.size());
  if (buf) {
    if (cap < n) return set_err(-22, "extradata buffer too small");
    std::memcpy(buf, c->extradata.data(), n);
  }
  return n;
}

int64_t ffv1hip_max_packet_size(const ffv1hip_ctx* c) { return c ? c->packet_stride : -22; }
int64_t ffv1hip_picture_number(const ffv1hip_ctx* c) { return c ? c->picture_number : -22; }
void ffv1hip_reset(ffv1hip_ctx* c) {
  if (c) {
    c->picture_number = 0;
    c->have_states = false;
  }
}

int ffv1hip_set_pass(ffv1hip_ctx* c, int pass, const char* stats_in) {
  if (!c || pass < 0 || pass > 2 || (pass == 2 && !stats_in)) return set_err(-22, "invalid arguments");
  if (c->picture_number || c->have_states || c->pass)
    return set_err(-22, "the pass is chosen once, before the first frame");
  if (pass == 0) return 0;
  const ffv1hip_params& p = c->P;
  if (p.version < 2) return set_err(-22, "2-pass needs version >= 2 (ffv1hip_options.pass)");
  HIP_TRY(hipSetDevice(c->device));
  if (pass == 1) {
    // the range coder's counts: from the decision stream in the
    // frame-parallel mode, by the chained coder as it codes otherwise
    // (context model 1, RGB, alpha, version 4); Golomb-Rice codes no range
    // decisions and writes zero counts, as the reference does
    const size_t bytes = sizeof(unsigned long long) * (512 + size_t(64) * c->contexts);
    HIP_TRY(hipMalloc(&c->d_rcstat, bytes));
    HIP_TRY(hipMalloc(&c->d_rcstat_bak, bytes));
    HIP_TRY(hipMemset(c->d_rcstat, 0, bytes));
    c->pass = 1;
    return 0;
  }
  uint8_t stt[256];
  std::memcpy(stt, c->frame.to1, 256);
  std::string err;
  const int rc = pass2_states(stats_in, p.ac == 2, stt, c->dflt.to1, c->init_states, &err);
  if (rc < 0) return set_err(rc, "%s", err.c_str());
  if (p.ac == 2) {  // the sorted table (ffv1enc.c:955-956), installed as in ffv1.c:95-101
    for (int i = 1; i < 256; i++) {
      c->frame.to1[i] = stt[i];
      c->frame.to0[256 - i] = uint8_t(256 - stt[i]);
    }
    HIP_TRY(hipMemcpy(c->d_tabs + 512, c->frame.to0, 256, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->d_tabs + 768, c->frame.to1, 256, hipMemcpyHostToDevice));
  }
  const std::vector<uint8_t>& is = c->init_states[p.context_model];
  HIP_TRY(hipMalloc(&c->d_init, is.size()));
  HIP_TRY(hipMemcpy(c->d_init, is.data(), is.size(), hipMemcpyHostToDevice));
  build_extradata(c);
  build_hdr(c);  // the slice header codes with the frame table
  const int urc = upload_hdr(c);
  if (urc < 0) return urc;
  c->pass = 2;
  return 0;
}

int64_t ffv1hip_stats_out(ffv1hip_ctx* c, char* buf, int64_t cap) {
  if (!c) return set_err(-22, "null ctx");
  if (c->pass != 1) return set_err(-22, "not a pass-1 context");
  HIP_TRY(hipSetDevice(c->device));
  const int rc = ffv1hip_synchronize(c);
  if (rc < 0) return rc;
  std::vector<uint64_t> h(512 + size_t(64) * c->contexts, 0);
  if (c->P.ac)
    HIP_TRY(hipMemcpy(h.data(), c->d_rcstat, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
  const std::string t = pass1_text(h.data(), h.data() + 512, c->contexts, c->P.context_model, int(c->gob_count));
  if (buf) {
    if (cap < int64_t(t.size()) + 1) return set_err(-22, "stats buffer too small");
    std::memcpy(buf, t.c_str(), t.size() + 1);
  }
  return int64_t(t.size());
}

// The sample width the residuals are folded / Golomb-coded at: RGB codes
// the transformed G', B' + off, R' + off with one more bit, 9 at 8 bit
// (ffv1enc.c:464-467).
static int coded_bits(const ffv1hip_params& p) {
  if (p.colorspace) return p.bits_per_raw_sample <= 8 ? 9 : p.bits_per_raw_sample + 1;
  return p.bits_per_raw_sample <= 8 ? 8 : p.bits_per_raw_sample;
}

// caller: the stream the frames were written on (their readiness is all the
// batch takes from it), or null when they are complete already.  The
// batch's own kernels run on the context's streams, so that a caller's
// stream never orders them after the previous batch's states walk.
static int run_batch(ffv1hip_ctx* c, const uint8_t* d_frames, int64_t frame_bytes,
                     const int64_t plane_off[kMaxPlanes], const int plane_stride[kMaxPlanes], int n, hipStream_t caller) {
  hipStream_t const st = c->stream;
  const ffv1hip_params& p = c->P;
  if (n <= 0 || n > c->max_batch) return set_err(-22, "batch of %d frames (max %d)", n, c->max_batch);
  // keyframes and state-chaining segments
  std::vector<uint8_t> keys(n);
  std::vector<Segment> segs;
  for (int i = 0; i < n; i++) {
    const int64_t pn = c->picture_number + i;
    keys[i] = uint8_t(p.gop_size == 0 || pn % p.gop_size == 0);
    if (i == 0 || keys[i]) segs.push_back(Segment{i, 0, 0, 0});
    segs.back().nframes++;
  }
  if (!keys[0] && !c->have_states)
    return set_err(-22, "P-frame without preceding keyframe state");
  segs.front().load_states = !keys[0];
  segs.back().save_states = 1;
  const int nsegs = int(segs.size());
  if (nsegs > c->max_slots) return set_err(-22, "batch spans %d GOPs (max %d)", nsegs, c->max_slots);
  // what to restore if this batch has to be encoded again (ffv1hip_fetch)
  ffv1hip_ctx::LastBatch& L = c->hist[c->nsub & 1];
  L.valid = true;
  L.frames = d_frames;
  L.frame_bytes = frame_bytes;
  const int nin = input_planes(p);
  for (int k = 0; k < kMaxPlanes; k++) {
    L.plane_off[k] = k < nin ? plane_off[k] : 0;
    L.plane_stride[k] = k < nin ? plane_stride[k] : 0;
  }
  L.n = n;
  L.st = caller;
  L.pn0 = c->picture_number;
  L.have0 = c->have_states;
  L.pcur0 = c->pcur;
  L.buf0 = c->buf;
  L.tri0 = c->tri;
  L.pk0 = c->pk;
  L.pk = c->two_pk ? c->pk : 0;
  L.gob0 = c->gob_count;
  L.keys.assign(keys.begin(), keys.end());
  for (uint8_t k : keys) c->gob_count += k;
  if (c->pass == 1) {
    // the previous batch's state counts (ffv1_stats_states, on the coder
    // stream) are in before the snapshot is taken
    if (c->dep_valid) HIP_TRY(hipStreamWaitEvent(st, c->done_ev, 0));
    HIP_TRY(hipMemcpyAsync(c->d_rcstat_bak, c->d_rcstat, sizeof(unsigned long long) * (512 + size_t(64) * c->contexts),
                           hipMemcpyDeviceToDevice, st));
  }
  // frames mode: the coder stream may still be on the previous batch, so the
  // buffers it reads alternate between two sets; set fb was last read by the
  // coder of batch k-2, which must be done before this batch rewrites it
  // (the stream metadata: three sets, t3)
  const int fb = c->buf;
  const int t3 = c->frames_mode ? c->tri : 0;
  uint8_t* const d_keys = c->frames_mode ? c->d_keys2 + size_t(t3) * c->max_batch : c->d_keys;
  // serial (measurement hook): no walk/code overlap
  const bool serial = c->knobs.has("serial");
  hipStream_t const cst = c->frames_mode && !serial ? c->code_stream : st;
  // the split schedule (two records sets): symbols, layout and bits on the
  // bits stream, beside the previous batch's walk
  hipStream_t const sst = c->frames_mode && c->two_rec && !serial ? c->bits_stream : st;
  if (caller) {  // the frames, for the symbols
    HIP_TRY(hipEventRecord(c->entry[fb], caller));
    HIP_TRY(hipStreamWaitEvent(st, c->entry[fb], 0));
    if (sst != st) HIP_TRY(hipStreamWaitEvent(sst, c->entry[fb], 0));
  }
  if (sst != st) {
    // what the symbols rewrite: records set fb (read by the walk of batch
    // k-2) and metadata set t3 (read by the coder of batch k-3)
    HIP_TRY(hipStreamWaitEvent(sst, c->walked[fb], 0));
    HIP_TRY(hipStreamWaitEvent(sst, c->coded3[t3], 0));
    // ... and start with the previous batch's walk: their bounded grids (no
    // LDS but a few hundred bytes per block) leave every CU the room its
    // three walk waves need, so the walk is never held back by them
    if (c->walk_a_valid) HIP_TRY(hipStreamWaitEvent(sst, c->walk_go, 0));
  }
  // the previous batch (possibly on another stream) is done with what this
  // one rewrites first: segments, slot lists, keyflags, the persist buffer
  if (c->dep_valid) HIP_TRY(hipStreamWaitEvent(st, c->dep_ev, 0));
  // (the walk rewrites decision-stream set fb: its last readers, range and
  // dseg of batch k-2, are done; the coder's join, bytes and packets after
  // them read none of it and run beside this walk)
  if (c->frames_mode) HIP_TRY(hipStreamWaitEvent(st, c->pre_read[fb], 0));
  HIP_TRY(hipMemcpyAsync(d_keys, keys.data(), n, hipMemcpyHostToDevice, sst));
  HIP_TRY(hipMemcpyAsync(c->d_segs, segs.data(), segs.size() * sizeof(Segment), hipMemcpyHostToDevice, st));

  int maxlen = 0;
  for (const Segment& g : segs) maxlen = std::max(maxlen, g.nframes);
  if (!c->frames_mode) {
    std::vector<int> slot_frames(size_t(maxlen) * nsegs, -1);
    for (int j = 0; j < maxlen; j++)
      for (int k = 0; k < nsegs; k++)
        if (j < segs[k].nframes) slot_frames[size_t(j) * nsegs + k] = segs[k].first_frame + j;
    HIP_TRY(hipMemcpyAsync(c->d_slot_frames, slot_frames.data(), sizeof(int) * slot_frames.size(),
                           hipMemcpyHostToDevice, st));
  }

  SymbolArgs sa{};
  sa.frames = d_frames;
  sa.frame_bytes = frame_bytes;
  // coded plane k: input plane k (YA8: Y and A both from input plane 0, one
  // byte apart, every second byte); context sets Y 0, Cb / Cr 1, A 2 (YA8's
  // A: 1), ffv1enc.c:1191-1201, (p + 1) / 2 for RGB (:460-467)
  const bool ya8 = is_ya8(p);
  for (int k = 0; k < kMaxPlanes; k++) {
    const int src = ya8 ? 0 : (k < nin ? k : 0);
    sa.plane_off[k] = plane_off[src] + (ya8 && k == 1 ? 1 : 0);
    sa.plane_stride[k] = plane_stride[src];
    sa.pstep[k] = ya8 ? 2 : 1;
    sa.pset[k] = ya8 ? k : (k + 1) / 2;
  }
  sa.nslots = nsegs;
  sa.geom = c->d_geom;
  sa.nslices = c->nslices;
  sa.nplanes = c->ncoded;
  sa.rct = c->d_rct;
  sa.sample_bytes = p.sample_bytes;
  sa.packed_at_lsb = p.packed_at_lsb;
  sa.msb_shift = 16 - p.bits_per_raw_sample;
  sa.coded_bits = coded_bits(p);
  sa.rgb = p.colorspace;
  sa.rct_offset = 1 << p.bits_per_raw_sample;
  sa.contexts = c->contexts;
  sa.model1 = p.context_model;
  sa.qt = c->frames_mode && c->d_qt_walk ? c->d_qt_walk : c->d_qt;
  uint32_t* const d_sym = c->frames_mode ? nullptr : c->d_sym;
  // walk records / chunk bits: set fb when there are two sets
  const bool rec1 = c->frames_mode && c->two_rec && fb == 1;
  uint2* d_rec = c->frames_mode ? (rec1 ? c->d_rec2 : reinterpret_cast<uint2*>(c->d_sym)) : nullptr;
  uint32_t* d_cbits = rec1 ? c->d_cbits2 : c->d_cbits;
  int* const d_dcount = c->frames_mode ? c->d_dcount + size_t(t3) * 3 * c->max_batch * c->nslices : nullptr;
  int64_t* const d_dbase = c->frames_mode ? c->d_dbase + size_t(t3) * c->max_batch * c->nslices : nullptr;
  StreamSegs* const d_segs = c->frames_mode ? c->d_segs_info + size_t(t3) * c->max_batch * c->nslices : nullptr;
  int* const d_segtot = c->frames_mode ? c->d_seg_totals + 2 * t3 : nullptr;
  int* const d_wmap = c->frames_mode ? c->d_wmap + size_t(t3) * c->max_groups : nullptr;
  sa.sym = d_sym;
  sa.frame_samples = c->frame_samples;

  CodeArgs ca{};
  ca.sym = d_sym;
  ca.frame_samples = c->frame_samples;
  ca.geom = c->d_geom;
  ca.nslices = c->nslices;
  ca.nsegs = nsegs;
  ca.segs = c->d_segs;
  ca.keyflags = d_keys;
  ca.ops = c->d_ops;
  ca.nops = c->d_nops;
  ca.max_ops = c->max_ops;
  ca.tabs = c->d_tabs;
  ca.state_bytes = int64_t(c->pcount) * c->contexts * 32;
  ca.tables = c->d_tables;
  ca.persist_in = c->d_persist[c->pcur];
  ca.persist_out = c->d_persist[c->pcur ^ 1];
  // overflow report of this batch (per buffer set: the coder of the
  // previous batch may still write the other one)
  const int sset = c->frames_mode ? fb : L.pk;
  L.status_set = sset;
  ca.status = c->d_status + 4 * sset;
  ca.slice_out = c->d_slice_out;
  ca.slice_cap = c->slice_cap;
  ca.slice_stride = c->slice_stride;
  ca.slice_bytes = c->d_slice_bytes;
  ca.version = p.version;
  ca.coded_bits = coded_bits(p);
  ca.rgb = p.colorspace;
  ca.nplanes = c->ncoded;
  ca.pcount = c->pcount;
  ca.rct = c->d_rct;
  for (int k = 0; k < kMaxPlanes; k++) ca.pset[k] = sa.pset[k];
  // v4 range coder: the reference's slice buffers (a packet of 16384 + 12 w h
  // bytes, all of it for slice 0, 1 / slice_count each for the others,
  // ffv1enc.c:1281-1282, 1317-1322) and the samples for the PCM re-code
  ca.v4pcm = p.version > 3 && p.ac;
  ca.v4_cap0 = 16384 + int64_t(p.width) * p.height * 12;
  ca.v4_cap = ca.v4_cap0 / c->nslices;
  // (v4_cap0=bytes, test hook: a smaller buffer for slice 0 alone, so that it
  // re-codes as PCM too; the oracle's FFV1_ORACLE_V4_CAP0)
  if (c->knobs.has("v4_cap0")) ca.v4_cap0 = c->knobs.get("v4_cap0", 0);
  ca.frames = d_frames;
  ca.frame_bytes = frame_bytes;
  for (int k = 0; k < kMaxPlanes; k++) {
    ca.plane_off[k] = sa.plane_off[k];
    ca.plane_stride[k] = sa.plane_stride[k];
  }
  ca.sample_bytes = p.sample_bytes;
  ca.packed_at_lsb = p.packed_at_lsb;
  ca.msb_shift = 16 - p.bits_per_raw_sample;
  ca.pcm_bits = p.bits_per_raw_sample <= 8 ? 8 : p.bits_per_raw_sample;  // coded_bits without the RGB + 1
  ca.init = c->d_init;

  if (c->profiling) HIP_TRY(hipEventRecord(c->ev[0], st));
  // brackets one launch with events when profiling (kind: 0 symbols, 1 code, 2 states)
  auto timed = [&](int kind, hipStream_t st, auto&& launch) -> int {
    if (c->profiling) {
      while (c->kev.size() < size_t(2) * (c->nkev + 1)) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return -1;
        c->kev.push_back(e);
      }
      if (c->kev_kind.size() < size_t(c->nkev + 1)) c->kev_kind.resize(c->nkev + 1);
      c->kev_kind[c->nkev] = kind;
      if (hipEventRecord(c->kev[2 * c->nkev], st) != hipSuccess) return -1;
    }
    const int rc = launch();
    if (c->profiling) {
      if (hipEventRecord(c->kev[2 * c->nkev + 1], st) != hipSuccess) return -1;
      c->nkev++;
    }
    return rc;
  };
  if (c->frames_mode) {
    // symbols of every frame, the decision layout, the states walk, then all
    // (frame, slice) streams at once
    sa.frame_of_slot = c->d_ident;
    sa.nslots = n;
    sa.dcount = d_dcount;  // accumulated by the symbols blocks of each plane
    // sym_skip=k (measurement hook, valid only when every batch codes the
    // same frames from a keyframe, as bench.py's): from batch max(k, 6) on,
    // no symbols pass; the batch reuses the records and chunk bits of the
    // batch two back (set fb) and the counts of the batch three back (t3)
    const bool sym_skip = c->knobs.has("sym_skip") && c->batches_run >= std::max(6, c->knobs.get("sym_skip", 6));
    c->batches_run++;
    if (!sym_skip) HIP_TRY(hipMemsetAsync(d_dcount, 0, sizeof(int) * 3 * size_t(n) * c->nslices, sst));
    sa.rec = d_rec;
    sa.cbits = d_cbits;
    sa.cwords = c->cwords;
    // one set: the previous batch's bits kernel (its own stream) has read the chunk bits
    if (sst == st) HIP_TRY(hipStreamWaitEvent(st, c->bitsed[fb ^ 1], 0));
    sa.frame_chunks = c->frame_chunks;
    sa.max_blocks = c->grid_sym;
    sa.rowb = c->walk_rowb;
    if (!sym_skip && timed(0, sst, [&] { return launch_symbols(sa, sst); }) < 0)
      return set_err(-5, "symbols launch failed: %s", hipGetErrorString(hipGetLastError()));
    // this batch's decisions, estimated from the earlier batches' totals
    // (per frame, the largest of the other two metadata sets, + 1/8), before
    // its layout overwrites its own set's
    int64_t est = 0;
    for (int k = 0; k < 3; k++)
      if (k != t3 && c->tri_n[k] > 0) est = std::max(est, c->h_tot_map[k] / c->tri_n[k]);
    est = est ? est * n + est * n / 8 + int64_t(n) * c->nslices * kStreamSlack : 0;
    c->tri_n[t3] = n;
    if (timed(4, sst, [&] {
          return launch_layout(d_dcount, n * c->nslices, d_dbase, c->d_dtotal + t3, d_segs, d_segtot, d_wmap,
                               c->hd_tot_map + t3, sst);
        }) < 0)
      return set_err(-5, "layout launch failed: %s", hipGetErrorString(hipGetLastError()));
    // decisions of this batch: the worst case fits without asking the device;
    // else, when the estimate fits the set as it is, the batch launches
    // guarded (its kernels skip it if its total does not fit after all, and
    // it is encoded again at settle, ds_over) without waiting for its
    // layout: the host goes on staging the next batch meanwhile.  Pass 1
    // (one count snapshot) and the readback=1 hook always read the total back.
    int64_t need = int64_t(n) * c->frame_samples * c->wmax + int64_t(n) * c->nslices * kStreamSlack;
    bool guarded = false;
    // (the guard_skip test hook: every batch launches guarded with a set its
    // decisions never fit, so that its kernels skip it and it takes the
    // recovery path: status[3], settle, the read-back re-run)
    const bool force_skip = c->knobs.has("guard_skip") && c->pass != 1 && !c->no_guard_once;
    if (force_skip ||
        (need > c->dcap[fb] && est > 0 && est <= c->dcap[fb] && c->pass != 1 && !c->no_guard_once &&
         !c->knobs.has("readback"))) {
      guarded = true;
      need = std::min(need, c->dcap[fb]);
    }
    c->no_guard_once = false;
    if (need > c->dcap[fb]) {
      HIP_TRY(hipMemcpyAsync(c->h_dtotal + t3, c->d_dtotal + t3, sizeof(int64_t), hipMemcpyDeviceToHost, sst));
      HIP_TRY(hipStreamSynchronize(sst));
      need = c->h_dtotal[t3];
      if (need > c->dcap[fb]) {
        // set fb's previous coder must be done before its buffers go (only
        // then: waiting for it on every batch held this batch's walk behind
        // the previous batch's packet assembly)
        HIP_TRY(hipEventSynchronize(c->coded[fb]));
        if (ensure_decisions(c, fb, need, &d_rec, &d_cbits) < 0)
          return set_err(-12, "decision buffers for %lld decisions: %s", (long long)need, g_err);
        sa.rec = d_rec;
        sa.cbits = d_cbits;
        sa.cwords = c->cwords;
        ca.slice_out = c->d_slice_out;  // (alloc_rec2 may have lowered the budget)
        ca.slice_cap = c->slice_cap;
        ca.slice_stride = c->slice_stride;
      }
    }
    HIP_TRY(hipEventRecord(c->laid[fb], sst));  // the records and the stream layout: the walk may start
    if (sst != st) HIP_TRY(hipStreamWaitEvent(sst, c->pre_read[fb], 0));  // d_bits[fb]: range / dseg of batch k-2
    if (guarded) {
      if (launch_zero_bits(c->d_bits[fb], c->d_dtotal + t3, c->dcap[fb], sst) < 0)
        return set_err(-5, "zero launch failed: %s", hipGetErrorString(hipGetLastError()));
    } else {
      HIP_TRY(hipMemsetAsync(c->d_bits[fb], 0, size_t((need + 31) / 32) * 4, sst));
    }
    DecisionStream ds{d_dcount, d_dbase, c->d_pre[fb], c->d_bits[fb], guarded ? c->d_dtotal + t3 : nullptr,
                      force_skip ? int64_t(-1) : c->dcap[fb]};
    if (force_skip) c->guard_skips++;
    BitsArgs ba{};
    ba.cbits = sa.cbits;
    ba.cwords = c->cwords;
    ba.frame_chunks = c->frame_chunks;
    ba.geom = c->d_geom;
    ba.nslices = c->nslices;
    ba.nframes = n;
    ba.ds = ds;
    ba.max_blocks = c->grid_bits;
    // the bits run beside the walk, on their own stream (after the layout
    // and the memset with the split schedule); the coder waits for both
    hipStream_t const bst = sst != st ? sst : serial ? st : c->bits_stream;
    if (sst == st) HIP_TRY(hipEventRecord(c->laid[fb], st));  // after the bits memset
    if (bst != sst) HIP_TRY(hipStreamWaitEvent(bst, c->laid[fb], 0));
    if (sst != st) HIP_TRY(hipStreamWaitEvent(st, c->laid[fb], 0));
    if (timed(5, bst, [&] { return launch_bits(ba, bst); }) < 0)
      return set_err(-5, "bits launch failed: %s", hipGetErrorString(hipGetLastError()));
    HIP_TRY(hipEventRecord(c->bitsed[fb], bst));
    WalkArgs wa{};
    wa.rec = d_rec;
    wa.cbits = d_cbits;
    wa.cwords = c->cwords;
    wa.frame_chunks = c->frame_chunks;
    wa.frame_samples = c->frame_samples;
    wa.geom = c->d_geom;
    wa.nslices = c->nslices;
    wa.segs = c->d_segs;
    wa.ftab = c->d_tabs + 512;
    wa.state_bytes = ca.state_bytes;
    wa.persist_in = ca.persist_in;
    wa.persist_out = ca.persist_out;
    wa.ds = ds;
    wa.scratch = c->d_scratch;
    if (kBoundsCheck) {
      // (the bounds_shrink hook: a smaller decision buffer than the real
      // one, so that the checks must fire; the test of the debug build)
      ca.bnd.err = c->d_bounds;
      ca.bnd.pre_bytes = c->dcap[fb] >> c->knobs.get("bounds_shrink", 0);
      ca.bnd.out_bytes = c->slice_stride * c->nslices * c->max_batch;
      ca.bnd.persist_bytes = ca.state_bytes * c->nslices;
      wa.bnd = ca.bnd;
    }
    wa.force_multi = c->knobs.has("force_multi");
    // wave priorities: the coder's serial range pass above the walk when the
    // walk is one round of chains no longer than the coder's streams (dense
    // rows, every walk wave resident, chroma chains no longer than luma's:
    // c3, c5); else the walk above the rest (c2: many rounds; c4: Cb and Cr
    // share a context set, a chroma chain is twice luma's).  Measured: c3
    // 14.1 vs 13.1 Gpix/s, c2 12.3 vs 13.3, c4 6.03 vs 6.15 (walk 0 / range 3
    // vs walk 2 / range 0).  The walk_prio / range_prio hooks override.
    bool range_first = false;
    {
      const SliceGeom& g0 = c->geom[0];
      const bool chroma_long = 2 * int64_t(g0.pw[1]) * g0.ph[1] > int64_t(g0.pw[0]) * g0.ph[0];
      wa.rows = c->walk_rows;
      wa.rowb = c->walk_rowb;
      wa.per_short = walk_per_short(g0);
      const int resident = walk_resident(wa);
      wa.short_multi = walk_split_short(nsegs, c->nslices, wa.per_short, 4 * c->cus, resident);
      // (the walk_blocks=0 hook, and the split-launch test hook, keep one-wave blocks)
      wa.block_waves = c->knobs.get("walk_blocks", 1) && !c->knobs.has("walk_part_a")
                           ? walk_block_waves(nsegs, c->nslices, wa.per_short, wa.short_multi, wa.rows, wa.rowb, c->cus,
                                              c->lds_block)
                           : 1;
      if (c->knobs.has("hostdbg"))
        std::fprintf(stderr, "hostdbg: walk of %d segments: %d-wave blocks (%d B of LDS per block allowed)\n", nsegs,
                     wa.block_waves, c->lds_block);
      range_first = c->d_qt_walk && !chroma_long &&
                    walk_items(nsegs, c->nslices, wa.per_short, wa.short_multi) <= resident;
    }
    wa.prio = c->knobs.get("walk_prio", range_first ? 0 : 2);
    const int range_prio = c->knobs.get("range_prio", range_first ? 3 : 0);
    wa.init = c->d_init;
    wa.rows = c->walk_rows;
    wa.dense = c->d_qt_walk != nullptr;
    if (c->knobs.has("walktrace") && c->trace_n < ffv1hip_ctx::kTraceBatches) {
      const int items = walk_items(nsegs, c->nslices, wa.per_short, wa.short_multi);
      if (!c->d_trace) {
        c->trace_items = walk_items(c->max_slots, c->nslices, 1, c->max_slots);
        HIP_TRY(hipMalloc(&c->d_trace, sizeof(uint64_t) * kTraceWords * c->trace_items * ffv1hip_ctx::kTraceBatches));
        HIP_TRY(hipMemset(c->d_trace, 0, sizeof(uint64_t) * kTraceWords * c->trace_items * ffv1hip_ctx::kTraceBatches));
      }
      if (items <= c->trace_items) wa.trace = c->d_trace + size_t(kTraceWords) * c->trace_items * c->trace_n;
    }
    // walkdbg (measurement hook): per-block cycle split to stderr
    const bool walkdbg = c->knobs.has("walkdbg");
    uint64_t* d_dbg = nullptr;
    const int nblk = walk_items(nsegs, c->nslices, wa.per_short, wa.short_multi);
    const int nlong = nsegs * ((c->nslices + 1) / 2);
    if (walkdbg) {
      HIP_TRY(hipMalloc(&d_dbg, sizeof(uint64_t) * 4 * nblk));
      HIP_TRY(hipMemsetAsync(d_dbg, 0, sizeof(uint64_t) * 4 * nblk, st));
      wa.dbg = d_dbg;
    }
    // split schedule: the first part is what the CUs hold at once
    // (one launch measured slower, round 4); one timed region either way
    const int nitems = walk_items(nsegs, c->nslices, wa.per_short, wa.short_multi);
    // walk_part_a (test hook): the first part's waves
    const bool pa = c->knobs.has("walk_part_a");
    const int first = sst != st ? (pa ? c->knobs.get("walk_part_a", 0) : walk_resident(wa)) : 0;
    // ... and only when the second part leaves room on the CUs beside it
    // (at most 80 % of the resident slots: c5's 100 % ran slower in round 2)
    const bool two_parts = wa.block_waves == 1 && first > 0 && first < nitems &&
                           (pa || int64_t(nitems - first) * 100 <= int64_t(first) * 80);
    HIP_TRY(hipEventRecord(c->walk_go, st));
    if (timed(2, st, [&] {
          if (!two_parts) return launch_walk(wa, nsegs, st);
          if (launch_walk(wa, nsegs, st, 0, first) < 0) return -1;
          if (hipEventRecord(c->walk_a, st) != hipSuccess) return -1;
          return launch_walk(wa, nsegs, st, first, -1);
        }) < 0)
      return set_err(-5, "walk launch failed: %s", hipGetErrorString(hipGetLastError()));
    if (!two_parts) HIP_TRY(hipEventRecord(c->walk_a, st));
    if (wa.trace) {
      c->trace_first.push_back(two_parts ? first : 0);
      c->trace_n++;
    }
    // (two_rec: also when the second records set came with this batch's layout)
    c->walk_a_valid = c->two_rec && !serial;
    StatsArgs sta{};
    if (c->pass == 1) {  // slot counts from the records, before the next batch's symbols rewrite them
      sta.rec = d_rec;
      sta.frame_samples = c->frame_samples;
      sta.geom = c->d_geom;
      sta.nslices = c->nslices;
      sta.nframes = n;
      sta.ds = ds;
      sta.rc_stat = c->d_rcstat;
      sta.rc_stat2 = c->d_rcstat + 512;
      sta.dense = c->d_qt_walk != nullptr;
      sta.rowb = c->walk_rowb;
      if (launch_stats(sta, false, st) < 0) return set_err(-5, "stats launch failed");
    }
    if (walkdbg) {
      std::vector<uint64_t> h(size_t(4) * nblk);
      HIP_TRY(hipMemcpyAsync(h.data(), d_dbg, h.size() * 8, hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      HIP_TRY(hipFree(d_dbg));
      double all[2] = {0, 0}, loop[2] = {0, 0}, steps[2] = {0, 0}, rt[2] = {0, 0};
      for (int b = 0; b < nblk; b++) {  // the longer plane group's chains first
        const int gi = b >= nlong;
        all[gi] += double(h[4 * b]);
        loop[gi] += double(h[4 * b + 1]);
        steps[gi] += double(h[4 * b + 2]);
        rt[gi] += double(h[4 * b + 3]);
      }
      for (int g = 0; g < 2; g++)
        std::fprintf(stderr, "walkdbg grp %d: blocks %d, memtime per block %.3g, loop share %.3f, memtime/step %.1f, "
                     "shader clock %.0f MHz, %.1f ns/step\n", g, g ? nblk - nlong : nlong, all[g] / (g ? nblk - nlong : nlong), loop[g] / all[g],
                     loop[g] / steps[g], all[g] / (rt[g] / 100.0), loop[g] / steps[g] / (all[g] / (rt[g] / 100.0)) * 1e3);
    }
    // the coder stream continues once this batch's walk is done; the walk of
    // the next batch (on st) then overlaps this batch's coding.  (Measured:
    // the range pass on a stream of its own, beside the previous batch's
    // dseg .. assembly, 11.0 Gpix/s against 17.6: with GPU_MAX_HW_QUEUES = 4
    // a fifth stream shares a hardware queue and serialises; 15.9 with 8.)
    HIP_TRY(hipEventRecord(c->walked[fb], st));
    HIP_TRY(hipStreamWaitEvent(cst, c->walked[fb], 0));
    HIP_TRY(hipStreamWaitEvent(cst, c->bitsed[fb], 0));
    if (c->pass == 1 && launch_stats(sta, true, cst) < 0) return set_err(-5, "stats launch failed");
    ca.nframes = n;
    ca.ds = ds;
    ca.hdr = c->d_hdr;
    ca.hdr_digits = c->d_hdr_digits;
    ca.segs_info = d_segs;
    ca.seg_totals = d_segtot;
    ca.wmap = d_wmap;
    ca.ck = c->d_ck;
    ca.segrec = c->d_segrec;
    ca.digit_cap = c->slice_stride / 4;
    ca.dseg_blocks = int(std::min<int64_t>(c->max_groups, c->grid_dseg));
    ca.range_prio = range_prio;
    ca.dseg_prio = c->prio_dseg;
    HIP_TRY(hipMemsetAsync(ca.status, 0, sizeof(int) * 4, cst));
    // range alone (the serial chain), every segment from its checkpoint,
    // the segments joined, then the bytes.  Split at the luma / chroma
    // boundary, the luma segments' dseg runs beside the chroma chains' range
    // pass in one launch, so the coder stream is range(luma) +
    // max(range(chroma), dseg(luma)) + dseg(chroma) instead of range + dseg
    // (the unsplit pass measured slower, round 4; its hook is gone).
    // (Timing: the fused launch counts as dseg.)
    ca.rstate = c->d_rstate;
    ca.range_pass = 1;
    ca.dseg_part = -1;
    if (timed(1, cst, [&] { return launch_range(ca, cst); }) < 0)
      return set_err(-5, "range launch failed: %s", hipGetErrorString(hipGetLastError()));
    ca.range_pass = 2;
    {
      CodeArgs cf = ca;  // the fused launch's dseg grid
      cf.dseg_blocks = std::max(1, ca.dseg_blocks);
      if (timed(7, cst, [&] { return launch_range_dseg(cf, cst); }) < 0)
        return set_err(-5, "range / dseg launch failed: %s", hipGetErrorString(hipGetLastError()));
    }
    ca.dseg_part = 1;
    if (timed(7, cst, [&] { return launch_dseg(ca, cst); }) < 0)
      return set_err(-5, "dseg launch failed: %s", hipGetErrorString(hipGetLastError()));
    HIP_TRY(hipEventRecord(c->pre_read[fb], cst));
    if (timed(8, cst, [&] { return launch_dfix(ca, cst); }) < 0)
      return set_err(-5, "dfix launch failed: %s", hipGetErrorString(hipGetLastError()));
    if (timed(6, cst, [&] { return launch_sink(ca, cst); }) < 0)
      return set_err(-5, "sink launch failed: %s", hipGetErrorString(hipGetLastError()));
  } else {
    HIP_TRY(hipMemsetAsync(ca.status, 0, sizeof(int) * 4, st));
    if (p.version > 3) {  // every (frame, slice)'s RCT coefficients, before the symbols and headers
      RctArgs ra{};
      ra.frames = d_frames;
      ra.frame_bytes = frame_bytes;
      for (int k = 0; k < 3; k++) {
        ra.plane_off[k] = plane_off[k < nin ? k : 0];
        ra.plane_stride[k] = plane_stride[k < nin ? k : 0];
      }
      ra.sample_bytes = p.sample_bytes;
      ra.geom = c->d_geom;
      ra.nslices = c->nslices;
      ra.nframes = n;
      ra.rct = c->d_rct;
      if (launch_rct_params(ra, st) < 0) return set_err(-5, "rct launch failed");
    }
    // ffv1_code's chains per wave: the batch's chains spread over two waves
    // per CU (a symbol costs a wave its chains' largest exponent, and few
    // chains at 64 per wave leave the SIMDs idle).  Measured (one box each,
    // tools/bench_chained.py): bgr0 1080p 480 chains 95 -> 132 Mpix/s (1 per
    // wave); ctx1 4K 1280 chains 445 (64) / 453 (2) / 479 (3); 5120 chains
    // 1,731 (64) / 1,732 (16) / 1,772 (10), but 1,587 at 7 (732 waves:
    // three per CU lose).  The code_cpw hook overrides (64: the round-5 form).
    ca.table_dummy = c->table_dummy;
    {
      const int64_t chains = int64_t(nsegs) * c->nslices, waves = int64_t(2) * std::max(1, c->cus);
      ca.cpw = (int)std::min<int64_t>(64, std::max<int64_t>(1, (chains + waves - 1) / waves));
      // the Golomb coder (no exponent-wide step) gains only from idle SIMDs:
      // c1 CIF 600 chains 529 -> 592 Mpix/s at 2 per wave, 1080p 5,760
      // chains 4,906 (64) -> 4,720 (12)
      if (!p.ac && chains > 4 * waves) ca.cpw = 64;
      ca.cpw = std::min(64, std::max(1, c->knobs.get("code_cpw", ca.cpw)));
    }
    for (int j = 0; j < maxlen; j++) {
      sa.frame_of_slot = c->d_slot_frames + size_t(j) * nsegs;
      if (timed(0, st, [&] { return launch_symbols(sa, st); }) < 0)
        return set_err(-5, "symbols launch failed: %s", hipGetErrorString(hipGetLastError()));
      ca.j = j;
      if (c->pass == 1 && p.ac) {
        ca.rc_stat = c->d_rcstat;
        ca.rc_stat2 = c->d_rcstat + 512;
      }
      if (timed(1, st, [&] { return p.ac ? launch_code(ca, st) : launch_code_golomb(ca, st); }) < 0)
        return set_err(-5, "code launch failed: %s", hipGetErrorString(hipGetLastError()));
    }
  }
  c->last_nsegs = c->frames_mode ? n : nsegs;

  AssembleArgs b{};
  b.skip = c->frames_mode ? ca.status + 3 : nullptr;
  b.slice_out = c->d_slice_out;
  b.slice_cap = c->slice_cap;
  b.slice_stride = c->slice_stride;
  b.slice_bytes = c->d_slice_bytes;
  b.packets = c->pkts(L.pk);
  b.packet_stride = c->packet_stride;
  b.packet_size = c->psize(L.pk);
  b.nslices = c->nslices;
  b.version = p.version;
  b.ec = p.ec;
  if (c->profiling) HIP_TRY(hipEventRecord(c->ev[1], cst));
  if (timed(3, cst, [&] { return launch_assemble(b, n, cst); }) < 0) return set_err(-5, "assemble launch failed");
  if (c->profiling) HIP_TRY(hipEventRecord(c->ev[2], cst));
  if (c->pipe.on) {  // the host-frame path then collects the batch with one D2H copy and no GPU work
    ffv1hip_ctx::HostPipe& P = c->pipe;
    if (launch_sizes_out(c->psize(L.pk), n, P.hd_sizes[L.pk], cst) < 0 ||
        launch_compact_packets(c->pkts(L.pk), c->packet_stride, c->psize(L.pk), n, P.d_compact[L.pk], b.skip, cst) < 0 ||
        launch_ints_out(ca.status, 4, P.hd_status + 4 * sset, cst) < 0)
      return set_err(-5, "collect launch failed: %s", hipGetErrorString(hipGetLastError()));
  }
  if (c->frames_mode) {
    HIP_TRY(hipEventRecord(c->coded[fb], cst));
    HIP_TRY(hipEventRecord(c->coded3[t3], cst));
    c->buf ^= 1;
    c->tri = (c->tri + 1) % 3;
  }
  HIP_TRY(hipEventRecord(c->dep_ev, st));  // frames mode: after the states walk
  HIP_TRY(hipEventRecord(c->done_ev, cst));
  c->dep_valid = true;
  c->pcur ^= 1;

  c->picture_number += n;
  c->have_states = true;
  HIP_TRY(hipEventRecord(c->hist_done[c->nsub & 1], cst));
  if (c->two_pk) c->pk ^= 1;
  c->nsub++;
  return 0;
}

int ffv1hip_encode_device(ffv1hip_ctx* c, const void* d_frames, int64_t frame_bytes,
                          const int64_t plane_offset[4], const int plane_stride[4], int n_frames,
                          void* stream) {
  if (!c || !d_frames) return set_err(-22, "null argument");
  HIP_TRY(hipSetDevice(c->device));
  return run_batch(c, static_cast<const uint8_t*>(d_frames), frame_bytes, plane_offset, plane_stride,
                   n_frames, reinterpret_cast<hipStream_t>(stream));
}

// A slice went over the byte budget: the reference would still have coded
// it (its buffer is ~w*h*140 bytes, ffv1enc.c:1232), so the batch is rolled
// back (picture number, P-frame carry, buffer sets) and encoded again with a
// budget sized from what the slice needed.  The batch's input frames must
// still be where the call found them.
static int alloc_compact(ffv1hip_ctx* c);
static int grow_slice_budget(ffv1hip_ctx* c, int64_t needed) {
  const int64_t cap = ((needed + needed / 4 + 4096) + 255) & ~int64_t(255);
  if (cap <= c->slice_cap) return set_err(-28, "slice byte budget %lld not enough", (long long)c->slice_cap);
  HIP_TRY(hipDeviceSynchronize());
  for (uint8_t** q : {&c->d_slice_out, &c->d_packets, &c->d_packets2}) {
    if (*q) HIP_TRY(hipFree(*q));
    *q = nullptr;
  }
  c->slice_cap = cap;
  c->slice_stride = c->frames_mode ? slice_stride_frames(cap) : cap;
  c->packet_stride = ((cap + 16) * c->nslices + 255) & ~int64_t(255);
  const size_t pk_bytes = size_t(c->packet_stride) * c->max_batch;
  for (int attempt = 0;; attempt++) {
    if (hipMalloc(&c->d_slice_out, size_t(c->slice_stride) * c->nslices * c->max_batch) == hipSuccess &&
        hipMalloc(&c->d_packets, pk_bytes) == hipSuccess &&
        (!c->two_pk || hipMalloc(&c->d_packets2, pk_bytes) == hipSuccess))
      break;
    (void)hipGetLastError();
    for (uint8_t** q : {&c->d_slice_out, &c->d_packets, &c->d_packets2}) {
      if (*q) HIP_TRY(hipFree(*q));
      *q = nullptr;
    }
    if (attempt > 0 || !c->two_rec) return set_err(-12, "slice buffers for a %lld-byte budget", (long long)cap);
    // the batches are rolled back (nothing in flight): the second records
    // set makes room, and the context goes on with one
    HIP_TRY(hipFree(c->d_rec2));
    HIP_TRY(hipFree(c->d_cbits2));
    c->d_rec2 = nullptr;
    c->d_cbits2 = nullptr;
    c->two_rec = false;
  }
  return c->pipe.on ? alloc_compact(c) : 0;
}

// Once batch b (one of the last two submitted) is done: if a slice of it
// went over the byte budget, roll it back and encode it again with a larger
// budget, then encode the batch submitted after it again too (it carried
// b's P-frame states and may use b's buffer sets), so that no caller ever
// sees a truncated slice (the reference fails a frame it cannot fit,
// ffv1enc.c:283-292; its buffer is large enough for any slice, :1232).
// Every batch reports into its own status set, cleared when the batch
// starts; the last two batches' sets are intact.
static const char* bounds_site(uint32_t s) {
  switch (s) {
    case kBndWalkStage: return "ffv1_walk (a chunk's recorded states)";
    case kBndWalkLong: return "ffv1_walk (a long chunk's recorded states)";
    case kBndWalkStates: return "ffv1_walk (the carried states)";
    case kBndDsegSlot: return "ffv1_dseg (a stream's digits)";
    case kBndDsegRead: return "ffv1_dseg (a segment's states, read)";
    case kBndDfixSlot: return "ffv1_dfix (a stream's digits)";
    case kBndSinkSlot: return "ffv1_sink (a stream's bytes)";
    default: return "an unknown site";
  }
}

static int settle_batch(ffv1hip_ctx* c, int64_t b) {
  if (b < 0 || b < c->nsub - 2 || b >= c->nsub) return 0;
  bool redo_next = false;
  bool pcm_fail = false;
  ffv1hip_ctx::LastBatch next;
  // re-runs: a slice over the byte budget (status[0]) grows the budget, at
  // most twice; a guarded batch whose decisions did not fit its set
  // (status[3], the kernels skipped it) runs once more with its total read
  // back, which cannot be skipped again, so it gets its own count
  int budget_runs = 0, set_runs = 0;
  for (;;) {
    const ffv1hip_ctx::LastBatch& L = c->hist[b & 1];
    HIP_TRY(hipEventSynchronize(c->hist_done[b & 1]));
    if (kBoundsCheck && c->d_bounds) {
      uint32_t site = 0;
      HIP_TRY(hipMemcpy(&site, c->d_bounds, sizeof(site), hipMemcpyDeviceToHost));
      if (site) return set_err(-14, "device bounds check: %s wrote outside its extent (debug build)", bounds_site(site));
    }
    int status[4];
    if (c->pipe.on) {
      // on the host-frame path a DMA copy would queue behind the next batch's
      // frames: a kernel writes the status into mapped host memory
      std::memcpy(status, c->pipe.h_status + 4 * L.status_set, sizeof(status));
    } else {
      HIP_TRY(hipMemcpy(status, c->d_status + 4 * L.status_set, sizeof(status), hipMemcpyDeviceToHost));
    }
    pcm_fail = status[2] != 0;
    if (!status[0] && !status[3]) break;
    if (!L.valid || (status[0] && budget_runs >= 2) || (status[3] && set_runs >= 1)) {
      if (status[3])
        return set_err(-28, "batch %lld: its decisions did not fit the decision set of a guarded launch, "
                            "even when encoded again with the total read back", (long long)b);
      return set_err(-28, "%d slices exceeded the slice byte budget", status[0]);
    }
    if (status[3]) {
      set_runs++;
      c->guard_reruns++;
    } else {
      budget_runs++;
    }
    if (!redo_next && b + 1 < c->nsub) {
      // pass 1 keeps one count snapshot, from before the last batch
      if (c->pass == 1) return set_err(-28, "pass 1: a slice of batch %lld went over the byte budget after a "
                                            "later batch was submitted", (long long)b);
      next = c->hist[(b + 1) & 1];
      redo_next = true;
    }
    HIP_TRY(hipDeviceSynchronize());
    const ffv1hip_ctx::LastBatch R = L;  // run_batch rewrites the slot
    c->picture_number = R.pn0;
    c->have_states = R.have0;
    c->pcur = R.pcur0;
    c->buf = R.buf0;
    c->tri = R.tri0;
    c->pk = R.pk0;
    c->walk_a_valid = false;
    c->gob_count = R.gob0;
    if (c->pass == 1)
      HIP_TRY(hipMemcpy(c->d_rcstat, c->d_rcstat_bak, sizeof(unsigned long long) * (512 + size_t(64) * c->contexts),
                        hipMemcpyDeviceToDevice));
    c->dep_valid = false;  // synchronised above
    c->nsub = b;
    int rc = status[0] ? grow_slice_budget(c, status[1]) : 0;
    if (rc < 0) return rc;
    // a guarded launch whose decisions did not fit its set (status[3]): sized
    // from its read-back total this time
    if (status[3]) c->no_guard_once = true;
    rc = run_batch(c, R.frames, R.frame_bytes, R.plane_off, R.plane_stride, R.n, nullptr);
    if (rc < 0) return rc;
  }
  if (redo_next) {
    const int rc = run_batch(c, next.frames, next.frame_bytes, next.plane_off, next.plane_stride, next.n, nullptr);
    if (rc < 0) return rc;
  }
  if (pcm_fail)  // the chained coder's v4 PCM re-code did not fit either
    return set_err(-38, "version 4: a slice overflowed its buffer even as PCM (the reference asserts there, "
                        "ffv1enc.c:1209)");
  return 0;
}

int ffv1hip_fetch(ffv1hip_ctx* c, uint8_t* out, int64_t out_cap, int64_t* sizes, int* key_flags) {
  if (!c) return set_err(-22, "null ctx");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipDeviceSynchronize());
  const int rc = settle_batch(c, c->nsub - 1);
  if (rc < 0) return rc;
  if (!c->nsub) return 0;
  const ffv1hip_ctx::LastBatch& L = c->last();
  const int n = L.n;
  std::vector<int64_t> sz(n);
  HIP_TRY(hipMemcpy(sz.data(), c->psize(L.pk), sizeof(int64_t) * n, hipMemcpyDeviceToHost));
  int64_t pos = 0;
  for (int i = 0; i < n; i++) {
    if (out) {
      if (pos + sz[i] > out_cap) return set_err(-22, "output buffer too small");
      HIP_TRY(hipMemcpy(out + pos, c->pkts(L.pk) + int64_t(i) * c->packet_stride, sz[i], hipMemcpyDeviceToHost));
    }
    pos += sz[i];
    if (sizes) sizes[i] = sz[i];
    if (key_flags) key_flags[i] = L.keys[i];
  }
  return 0;
}

int ffv1hip_synchronize(ffv1hip_ctx* c) {
  if (!c) return set_err(-22, "null ctx");
  HIP_TRY(hipSetDevice(c->device));
  if (c->dep_valid) HIP_TRY(hipEventSynchronize(c->done_ev));  // also a caller-given launch stream
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (c->code_stream) HIP_TRY(hipStreamSynchronize(c->code_stream));
  if (c->bits_stream) HIP_TRY(hipStreamSynchronize(c->bits_stream));
  return settle_batch(c, c->nsub - 1);
}

int ffv1hip_device_packets(ffv1hip_ctx* c, void** d_packets, int64_t* packet_stride, void** d_sizes) {
  if (!c) return set_err(-22, "null ctx");
  // the packets are only valid once settled; a re-encode may also move them
  const int rc = ffv1hip_synchronize(c);
  if (rc < 0) return rc;
  const int pk = c->nsub ? c->last().pk : 0;
  if (d_packets) *d_packets = c->pkts(pk);
  if (packet_stride) *packet_stride = c->packet_stride;
  if (d_sizes) *d_sizes = c->psize(pk);
  return 0;
}

// Where the planes of one frame sit in a batch slot of d_frames (tightly
// packed rows): np planes, plane k at off[k] with rows[k] rows of pst[k]
// bytes.  bgr0 is one packed plane.
static void slot_layout(const ffv1hip_ctx* c, int64_t off[kMaxPlanes], int pst[kMaxPlanes], int rows[kMaxPlanes],
                        int* np) {
  const ffv1hip_params& p = c->P;
  const int cw = -((-p.width) >> p.chroma_h_shift), ch = -((-p.height) >> p.chroma_v_shift);
  *np = input_planes(p);
  off[0] = 0;
  off[1] = c->plane_bytes[0];
  off[2] = c->plane_bytes[0] + c->plane_bytes[1];
  off[3] = off[2] + c->plane_bytes[2];
  pst[0] = p.width * p.sample_bytes * (is_ya8(p) ? 2 : 1);
  pst[1] = pst[2] = cw * p.sample_bytes;
  pst[3] = p.width * p.sample_bytes;
  rows[0] = rows[3] = p.height;
  rows[1] = rows[2] = ch;
}

// ---------------------------------------------------------------------------
// The host-frame path (ffv1hip_encode, ffv1hip_encode2).  On first use: the
// batch's frame slots (not needed by ffv1hip_encode_device), the transfer
// stream, the pinned staging slots and the copy threads; and, with HBM to
// spare and outside pass 1, a second frame set and a second packet set, so
// that batch k+1's frames are copied in while batch k codes and batch k-1's
// packets are copied out (PCIe both ways beside the kernels).
// The packed packets of a packet set: the worst case, a full set.
static int alloc_compact(ffv1hip_ctx* c) {
  ffv1hip_ctx::HostPipe& P = c->pipe;
  const int64_t cap = c->packet_stride * c->max_batch;
  for (int k = 0; k < (c->two_pk ? 2 : 1); k++) {
    if (P.d_compact[k]) HIP_TRY(hipFree(P.d_compact[k]));
    P.d_compact[k] = nullptr;
    if (hipMalloc(&P.d_compact[k], size_t(cap)) != hipSuccess) {
      (void)hipGetLastError();
      return set_err(-12, "packed packets of a %d-frame batch (%.1f GB) do not fit in device memory", c->max_batch,
                     double(cap) / 1e9);
    }
    P.d_compact_cap[k] = cap;
  }
  return 0;
}

static void pipe_release(ffv1hip_ctx* c);

// The second frame / packet set of the overlapped host path, freed.
static void drop_second_set(ffv1hip_ctx* c) {
  (void)hipGetLastError();
  for (void** q : {(void**)&c->d_frames2, (void**)&c->d_frames3, (void**)&c->d_packets2,
                   (void**)&c->d_packet_size2}) {
    if (*q) (void)hipFree(*q);
    *q = nullptr;
  }
  c->two_pk = false;
  c->pipe.overlap = false;
  c->pipe.nsets = 1;
}

static int pipe_open_parts(ffv1hip_ctx* c) {
  ffv1hip_ctx::HostPipe& P = c->pipe;
  const size_t fset = size_t(c->frame_bytes) * c->max_batch;
  if (!c->d_frames && hipMalloc(&c->d_frames, fset) != hipSuccess) {
    (void)hipGetLastError();
    c->d_frames = nullptr;
    return set_err(-12, "the frame slots of a %d-frame batch (%.1f GB) do not fit in device memory", c->max_batch,
                   double(fset) / 1e9);
  }
  {
    // both copy streams at the greatest priority: a queue pool of their own,
    // so that the host path fits the runtime's default 4 hardware queues
    // (at default priority the packets-out stream shared the walk stream's
    // queue: encode2 batch 240 7,132 -> 8,383 Mpix/s, gpurun_out/r5l)
    int lo = 0, hi = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIP_TRY(hipStreamCreateWithPriority(&P.xfer, hipStreamNonBlocking, hi));
    HIP_TRY(hipStreamCreateWithPriority(&P.d2h, hipStreamNonBlocking, hi));
  }
  int nt = int(std::thread::hardware_concurrency());
  if (const char* e = std::getenv("OMP_NUM_THREADS"))  // the host's CPU share where it is set
    if (std::atoi(e) > 0) nt = std::min(nt, std::atoi(e));
  nt = c->knobs.get("copy_threads", nt);
  P.pool = std::make_unique<CopyPool>(std::max(1, std::min(nt, 16)));
  P.pool_out = std::make_unique<CopyPool>(std::max(1, std::min(nt / 4, 4)));
  P.dbg = c->knobs.has("hostdbg");
  P.slot_bytes = std::max<int64_t>(int64_t(32) << 20, int64_t(c->P.width) * 4);
  for (int k = 0; k < ffv1hip_ctx::HostPipe::kSlots; k++) {
    HIP_TRY(hipHostMalloc(&P.h_slot[k], size_t(P.slot_bytes), hipHostMallocDefault));
    HIP_TRY(hipEventCreateWithFlags(&P.slot_ev[k], hipEventDisableTiming));
  }
  if (c->pass != 1) {
    // the second set: frames, packets, their sizes, and the second packed
    // packets buffer alloc_compact adds (with the first one, not allocated
    // yet either), with 2 GB to spare
    size_t free_b = 0, total_b = 0;
    HIP_TRY(hipMemGetInfo(&free_b, &total_b));
    const size_t pk_bytes = size_t(c->packet_stride) * c->max_batch;
    if (free_b > fset + 3 * pk_bytes + (size_t(2) << 30) && hipMalloc(&c->d_frames2, fset) == hipSuccess &&
        hipMalloc(&c->d_packets2, pk_bytes) == hipSuccess &&
        hipMalloc(&c->d_packet_size2, sizeof(int64_t) * c->max_batch) == hipSuccess) {
      HIP_TRY(hipMemset(c->d_packet_size2, 0, sizeof(int64_t) * c->max_batch));
      c->two_pk = true;
      P.overlap = true;
      P.nsets = 2;
      // a third frame set with room to spare (fsets=2: two)
      if (c->knobs.get("fsets", 3) >= 3 && free_b > 2 * fset + 3 * pk_bytes + (size_t(4) << 30)) {
        if (hipMalloc(&c->d_frames3, fset) == hipSuccess) {
          P.nsets = 3;
        } else {
          (void)hipGetLastError();
          c->d_frames3 = nullptr;
        }
      }
    } else {
      drop_second_set(c);
    }
  }
  {  // 10-bit samples packed for PCIe (pack=0: as they are)
    const ffv1hip_params& p = c->P;
    P.pack10 = p.sample_bytes == 2 && p.packed_at_lsb && p.bits_per_raw_sample == 10 && !is_ya8(p) &&
               c->knobs.get("pack", 1) != 0;
    if (P.pack10) {
      int64_t off[kMaxPlanes];
      int pst[kMaxPlanes], rows[kMaxPlanes], np;
      slot_layout(c, off, pst, rows, &np);
      int64_t o = 0;
      for (int k = 0; k < np; k++) {
        P.poff[k] = o;
        P.pw[k] = pst[k] / 2;
        P.prow[k] = (P.pw[k] + 2) / 3 * 4;
        o += int64_t(P.prow[k]) * rows[k];
      }
      P.packed_frame_bytes = (o + 255) & ~int64_t(255);
      for (int k = 0; k < P.nsets && P.pack10; k++) {
        if (hipMalloc(&P.d_packed[k], size_t(P.packed_frame_bytes) * c->max_batch) != hipSuccess) {
          (void)hipGetLastError();
          P.d_packed[k] = nullptr;
          P.pack10 = false;  // (the frames go as they are)
        }
        P.rawf[k].assign(size_t(c->max_batch), 1);
      }
      if (!P.pack10)
        for (uint8_t*& d : P.d_packed) {
          if (d) (void)hipFree(d);
          d = nullptr;
        }
    }
  }
  for (int k = 0; k < 2; k++) {  // both packet sets' mapped sizes (the second may come into use)
    HIP_TRY(hipHostMalloc(&P.h_sizes[k], sizeof(int64_t) * size_t(c->max_batch), hipHostMallocMapped));
    HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&P.hd_sizes[k]), P.h_sizes[k], 0));
  }
  HIP_TRY(hipHostMalloc(&P.h_status, sizeof(int) * 8, hipHostMallocMapped));
  HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&P.hd_status), P.h_status, 0));
  int rc = alloc_compact(c);
  if (rc < 0 && P.overlap) {  // one set then: the second one's memory goes to the packed packets
    for (uint8_t*& d : P.d_compact) {
      if (d) (void)hipFree(d);
      d = nullptr;
    }
    drop_second_set(c);
    rc = alloc_compact(c);
  }
  return rc;
}

// On first use of the host-frame path; a failure part way releases what it
// had set up, so a later call starts from scratch.
static int pipe_open(ffv1hip_ctx* c) {
  if (c->pipe.on) return 0;
  const int rc = pipe_open_parts(c);
  if (rc < 0) {
    const std::string err = g_err;
    pipe_release(c);
    return set_err(rc, "%s", err.c_str());
  }
  c->pipe.on = true;
  return 0;
}

static void pipe_close(ffv1hip_ctx* c) {
  ffv1hip_ctx::HostPipe& P = c->pipe;
  if (P.xfer) (void)hipStreamSynchronize(P.xfer);
  P.pool.reset();
  P.pool_out.reset();
  for (int k = 0; k < ffv1hip_ctx::HostPipe::kSlots; k++) {
    if (P.h_slot[k]) (void)hipHostFree(P.h_slot[k]);
    if (P.slot_ev[k]) (void)hipEventDestroy(P.slot_ev[k]);
  }
  for (uint8_t* h : P.h_pk)
    if (h) (void)hipHostFree(h);
  for (int64_t* h : P.h_sizes)
    if (h) (void)hipHostFree(h);
  if (P.h_status) (void)hipHostFree(P.h_status);
  for (uint8_t* d : P.d_compact)
    if (d) (void)hipFree(d);
  for (uint8_t* d : P.d_packed)
    if (d) (void)hipFree(d);
  if (P.xfer) (void)hipStreamDestroy(P.xfer);
  if (P.d2h) (void)hipStreamDestroy(P.d2h);
  for (void* q : {(void*)c->d_frames2, (void*)c->d_frames3, (void*)c->d_packets2, (void*)c->d_packet_size2})
    if (q) (void)hipFree(q);
  c->d_frames2 = nullptr;
  c->d_frames3 = nullptr;
  c->d_packets2 = nullptr;
  c->d_packet_size2 = nullptr;
}

// pipe_close, and the pipe back to its unopened state
static void pipe_release(ffv1hip_ctx* c) {
  pipe_close(c);
  c->pipe.~HostPipe();
  new (&c->pipe) ffv1hip_ctx::HostPipe();
  c->two_pk = false;
  (void)hipGetLastError();
}

// The current staging slot's copies are all queued: mark it busy until they
// are done.
static int stage_flush(ffv1hip_ctx* c) {
  ffv1hip_ctx::HostPipe& P = c->pipe;
  if (P.fill == 0) return 0;
  HIP_TRY(hipEventRecord(P.slot_ev[P.next], P.xfer));
  P.slot_busy[P.next] = true;
  P.next = (P.next + 1) % ffv1hip_ctx::HostPipe::kSlots;
  P.fill = 0;
  return 0;
}

// rows of wb bytes of a host plane (pitch sp) to device memory with tight
// rows at dst: piece by piece, copied into a pinned slot by the pool and
// sent with one async copy on the transfer stream; a slot is reused once
// its copies are done.
static bool host_registered(const ffv1hip_ctx* c, const void* p, int64_t n) {
  if (c->host_ranges.empty()) return false;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  auto it = c->host_ranges.upper_bound(a);
  if (it == c->host_ranges.begin()) return false;
  --it;
  return a + uintptr_t(n) <= it->first + uintptr_t(it->second.bytes);
}

static int stage_rows(ffv1hip_ctx* c, uint8_t* dst, const uint8_t* src, int64_t sp, int64_t wb, int64_t rows) {
  ffv1hip_ctx::HostPipe& P = c->pipe;
  if (rows > 0 && host_registered(c, src, (rows - 1) * sp + wb)) {  // caller-pinned: one DMA from it
    const double t0 = P.dbg ? wall_s() : 0;
    if (sp == wb)
      HIP_TRY(hipMemcpyAsync(dst, src, size_t(rows * wb), hipMemcpyHostToDevice, P.xfer));
    else
      HIP_TRY(hipMemcpy2DAsync(dst, size_t(wb), src, size_t(sp), size_t(wb), size_t(rows), hipMemcpyHostToDevice,
                               P.xfer));
    if (P.dbg) P.t_dma += wall_s() - t0;
    c->direct_pending = true;
    return 0;
  }
  for (int64_t r = 0; r < rows;) {
    if (P.fill + wb > P.slot_bytes) {
      const int rc = stage_flush(c);
      if (rc < 0) return rc;
    }
    double t0 = P.dbg ? wall_s() : 0;
    if (P.fill == 0 && P.slot_busy[P.next]) {
      HIP_TRY(hipEventSynchronize(P.slot_ev[P.next]));
      P.slot_busy[P.next] = false;
    }
    const int64_t nr = std::min(rows - r, (P.slot_bytes - P.fill) / wb);
    uint8_t* const h = P.h_slot[P.next] + P.fill;
    double t1 = P.dbg ? wall_s() : 0;
    pool_copy2d(*P.pool, h, wb, src + r * sp, sp, wb, nr);
    double t2 = P.dbg ? wall_s() : 0;
    HIP_TRY(hipMemcpyAsync(dst + r * wb, h, size_t(nr * wb), hipMemcpyHostToDevice, P.xfer));
    if (P.dbg) {
      const double t3 = wall_s();
      P.t_slot += t1 - t0;
      P.t_copy += t2 - t1;
      P.t_dma += t3 - t2;
    }
    P.fill += nr * wb;
    r += nr;
  }
  return 0;
}

// stage_rows for 10-bit samples: rows of w samples packed into the pinned
// slots (pb bytes a row) and sent to the packed area at dst; *acc: the OR
// of the samples.
static int stage_rows_packed(ffv1hip_ctx* c, uint8_t* dst, const uint8_t* src, int64_t sp, int w, int64_t pb,
                             int64_t rows, uint32_t* acc) {
  ffv1hip_ctx::HostPipe& P = c->pipe;
  for (int64_t r = 0; r < rows;) {
    if (P.fill + pb > P.slot_bytes) {
      const int rc = stage_flush(c);
      if (rc < 0) return rc;
    }
    double t0 = P.dbg ? wall_s() : 0;
    if (P.fill == 0 && P.slot_busy[P.next]) {
      HIP_TRY(hipEventSynchronize(P.slot_ev[P.next]));
      P.slot_busy[P.next] = false;
    }
    const int64_t nr = std::min(rows - r, (P.slot_bytes - P.fill) / pb);
    uint8_t* const h = P.h_slot[P.next] + P.fill;
    double t1 = P.dbg ? wall_s() : 0;
    *acc |= pool_pack10(*P.pool, h, pb, src + r * sp, sp, w, nr);
    double t2 = P.dbg ? wall_s() : 0;
    HIP_TRY(hipMemcpyAsync(dst + r * pb, h, size_t(nr * pb), hipMemcpyHostToDevice, P.xfer));
    if (P.dbg) {
      const double t3 = wall_s();
      P.t_slot += t1 - t0;
      P.t_copy += t2 - t1;
      P.t_dma += t3 - t2;
    }
    P.fill += nr * pb;
    r += nr;
  }
  return 0;
}

// One host frame into batch slot `slot` of frame set `set`: packed (10-bit
// samples, none over 10 bits, not caller-pinned) or as it is.
static uint8_t* frame_set(const ffv1hip_ctx* c, int set) {
  return set == 0 ? c->d_frames : set == 1 ? c->d_frames2 : c->d_frames3;
}

static int stage_frame(ffv1hip_ctx* c, int set, int64_t slot, const void* const* planes, const int* strides) {
  ffv1hip_ctx::HostPipe& P = c->pipe;
  int64_t off[kMaxPlanes];
  int pst[kMaxPlanes], rows[kMaxPlanes], np;
  slot_layout(c, off, pst, rows, &np);
  for (int k = 0; k < np; k++)
    if (!planes[k]) return set_err(-22, "null plane %d", k);
  uint8_t* const base = frame_set(c, set) + slot * c->frame_bytes;
  bool raw = true;
  if (P.pack10 && P.d_packed[set]) {
    bool pinned = false;
    for (int k = 0; k < np; k++)
      pinned = pinned || (rows[k] > 0 && host_registered(c, planes[k], int64_t(rows[k] - 1) * strides[k] + pst[k]));
    if (!pinned) {
      uint8_t* const pbase = P.d_packed[set] + slot * P.packed_frame_bytes;
      uint32_t acc = 0;
      for (int k = 0; k < np && acc < 1024u; k++) {
        const int rc = stage_rows_packed(c, pbase + P.poff[k], static_cast<const uint8_t*>(planes[k]), strides[k],
                                         P.pw[k], P.prow[k], rows[k], &acc);
        if (rc < 0) return rc;
      }
      raw = acc >= 1024u;  // a sample over 10 bits: the frame goes as it is (the packed bytes unused)
    }
    P.rawf[set][size_t(slot)] = raw ? 1 : 0;
  }
  if (raw)
    for (int k = 0; k < np; k++) {
      const int rc = stage_rows(c, base + off[k], static_cast<const uint8_t*>(planes[k]), strides[k], pst[k], rows[k]);
      if (rc < 0) return rc;
    }
  return 0;
}

// Batch `set`'s queued frames (staged) as one batch.
static int launch_staged(ffv1hip_ctx* c, int set, int n) {
  int rc = stage_flush(c);
  if (rc < 0) return rc;
  int64_t off[kMaxPlanes];
  int pst[kMaxPlanes], rows[kMaxPlanes], np;
  slot_layout(c, off, pst, rows, &np);
  ffv1hip_ctx::HostPipe& P = c->pipe;
  uint8_t* const frames = frame_set(c, set);
  if (P.pack10 && P.d_packed[set]) {  // the packed frames into their slots, after their copies
    for (int f0 = 0; f0 < n; f0 += kUnpackFrames) {
      UnpackArgs ua{};
      ua.packed = P.d_packed[set];
      ua.frames = frames;
      ua.packed_frame_bytes = P.packed_frame_bytes;
      ua.frame_bytes = c->frame_bytes;
      ua.np = np;
      ua.f0 = f0;
      bool any = false;
      for (int k = 0; k < np; k++) {
        ua.poff[k] = P.poff[k];
        ua.off[k] = off[k];
        ua.prow[k] = P.prow[k] / 4;
        ua.width[k] = P.pw[k];
        ua.rows[k] = rows[k];
        ua.pst[k] = pst[k];
      }
      const int nf = std::min(kUnpackFrames, n - f0);
      for (int i = 0; i < nf; i++) {
        const bool r = P.rawf[set][size_t(f0 + i)] != 0;
        ua.raw[i >> 5] |= uint32_t(r) << (i & 31);
        any = any || !r;
      }
      if (any && launch_unpack10(ua, nf, P.xfer) < 0)
        return set_err(-5, "unpack launch failed: %s", hipGetErrorString(hipGetLastError()));
    }
  }
  return run_batch(c, frames, c->frame_bytes, off, pst, n, P.xfer);
}

// A settled batch's packets (n of them, packet set pk) into the pinned
// buffer of that set, on `st`: sizes, offsets and the buffer out.  Only
// reads the context's buffers, so the copy-out thread of ffv1hip_encode
// runs it beside the main thread's staging.
static int copy_packets(ffv1hip_ctx* c, int n, int pk, hipStream_t st, std::vector<int64_t>& sz,
                        std::vector<int64_t>& off, const uint8_t** data) {
  ffv1hip_ctx::HostPipe& P = c->pipe;
  sz.resize(n);
  off.resize(n);
  const double ts0 = P.dbg ? wall_s() : 0;
  std::memcpy(sz.data(), P.h_sizes[pk], sizeof(int64_t) * size_t(n));  // the batch is done (hist_done)
  if (P.dbg) P.t_sizes += wall_s() - ts0;
  int64_t total = 0;
  for (int i = 0; i < n; i++) {
    off[i] = total;
    total += sz[i];
  }
  if (total > P.h_pk_cap[pk]) {
    if (P.h_pk[pk]) HIP_TRY(hipHostFree(P.h_pk[pk]));
    P.h_pk[pk] = nullptr;
    P.h_pk_cap[pk] = 0;
    const int64_t cap = (total + total / 4 + (int64_t(1) << 20)) & ~int64_t(4095);
    HIP_TRY(hipHostMalloc(&P.h_pk[pk], size_t(cap), hipHostMallocDefault));
    P.h_pk_cap[pk] = cap;
  }
  uint8_t* const h = P.h_pk[pk];
  // one D2H copy of the packets the batch packed back to back (a copy per
  // packet runs at a few GB/s)
  const double tc1 = P.dbg ? wall_s() : 0;
  if (total) HIP_TRY(hipMemcpyAsync(h, P.d_compact[pk], size_t(total), hipMemcpyDeviceToHost, st));
  if (P.dbg) {
    HIP_TRY(hipStreamSynchronize(st));
    P.t_dcopy += wall_s() - tc1;
  }
  HIP_TRY(hipStreamSynchronize(st));
  *data = h;
  return 0;
}

// Batch b's packets (its slice budget settled first) into the pinned buffer
// of its packet set.
static int collect(ffv1hip_ctx* c, int64_t b, std::vector<int64_t>& sz, std::vector<int64_t>& off,
                   const uint8_t** data) {
  int rc = settle_batch(c, b);
  if (rc < 0) return rc;
  HIP_TRY(hipEventSynchronize(c->hist_done[b & 1]));
  const ffv1hip_ctx::LastBatch& L = c->hist[b & 1];
  return copy_packets(c, L.n, L.pk, c->pipe.d2h, sz, off, data);  // not behind the frames on xfer
}

int ffv1hip_encode(ffv1hip_ctx* c, const void* const* planes, const int* strides, int n_frames,
                   uint8_t* out, int64_t out_cap, int64_t* sizes, int* key_flags) {
  if (!c || !planes || !strides) return set_err(-22, "null argument");
  if (!c->q_pts.empty() || !c->launched.empty() || c->ready.next < c->ready.size.size())
    return set_err(-22, "ffv1hip_encode2 has frames or packets pending: flush it first");
  HIP_TRY(hipSetDevice(c->device));
  int rc = pipe_open(c);
  if (rc < 0) return rc;
  ffv1hip_ctx::HostPipe& P = c->pipe;
  int64_t used = 0;
  // Batch b's collector: once the batch is done on the GPU, its packets come
  // over PCIe into the pinned buffer of its packet set (a thread of its own,
  // started when the batch is launched, so that this thread only stages
  // frames).  It is joined two batches later, before batch b + 2 is staged
  // into b's frame set and launched into b's packet set; the packets then go
  // into `out` in batch order.  A batch over the slice byte budget is left to
  // that join: its frames are still in place for the re-encode.
  struct Out {
    std::thread th;
    int64_t b = -1;  // the batch, -1: none
    int base = 0, n = 0;
    bool redo = false;
    int rc = 0;
    std::string err;
    std::vector<int64_t> sz;
    std::vector<int> keys;
    const uint8_t* h = nullptr;
  } ot[2];
  auto collect_async = [&, c](Out& o, int64_t b, int base) {
    const ffv1hip_ctx::LastBatch& L = c->hist[b & 1];
    o.b = b;
    o.base = base;
    o.n = L.n;
    o.keys = L.keys;
    o.redo = false;
    o.rc = 0;
    const int pk = L.pk, sset = L.status_set;
    hipEvent_t const ev = c->hist_done[b & 1];
    o.th = std::thread([&o, &P, c, ev, pk, sset]() {
      const double t0 = wall_s();
      if (const hipError_t e = hipEventSynchronize(ev); e != hipSuccess) {
        o.rc = set_err(-5, "batch wait failed: %s", hipGetErrorString(e));
        o.err = g_err;
        return;
      }
      P.t_settle += wall_s() - t0;
      if (P.h_status[4 * sset] || P.h_status[4 * sset + 3]) {  // over the budget or the set: settled at the join
        o.redo = true;
        return;
      }
      std::vector<int64_t> off;
      const double t1 = wall_s();
      const int r = copy_packets(c, o.n, pk, P.d2h, o.sz, off, &o.h);
      P.t_d2h += wall_s() - t1;
      if (r < 0) {
        o.rc = r;
        o.err = g_err;
      }
    });
  };
  // the collected packets of o's batch into `out`
  auto deliver = [&](Out& o) -> int {
    int64_t total = 0;
    for (int64_t v : o.sz) total += v;
    if (out && used + total > out_cap) return set_err(-22, "output buffer too small");
    const double t0 = wall_s();
    if (out && total) pool_copy2d(*P.pool, out + used, total, o.h, total, total, 1);
    P.t_out += wall_s() - t0;
    for (int i = 0; i < o.n; i++) {
      if (sizes) sizes[o.base + i] = o.sz[i];
      if (key_flags) key_flags[o.base + i] = o.keys[i];
    }
    used += total;
    o.b = -1;
    return 0;
  };
  // a batch settled (re-encoded if need be) and collected on this thread
  auto collect_sync = [&](Out& o) -> int {
    int r = settle_batch(c, o.b);
    if (r < 0) return r;
    HIP_TRY(hipEventSynchronize(c->hist_done[o.b & 1]));
    const ffv1hip_ctx::LastBatch& L = c->hist[o.b & 1];
    o.keys = L.keys;
    std::vector<int64_t> off;
    return copy_packets(c, o.n, L.pk, P.d2h, o.sz, off, &o.h);
  };
  auto join = [&](Out& o) -> int {
    const double t0 = wall_s();
    if (o.th.joinable()) o.th.join();
    P.t_join += wall_s() - t0;
    return o.rc < 0 ? set_err(o.rc, "%s", o.err.c_str()) : 0;
  };
  // batch j - 2's collector (before batch j reuses its sets); a re-encode of
  // it also re-encodes batch j - 1, whose collector is then redone here
  auto retire = [&](int64_t b) -> int {
    Out& o = ot[b & 1];
    if (o.b != b) return 0;
    int r = join(o);
    if (r < 0) return r;
    if (o.redo) {
      Out& nx = ot[(b + 1) & 1];
      if (nx.b == b + 1) {
        if ((r = join(nx)) < 0) return r;
      }
      if ((r = collect_sync(o)) < 0) return r;
      if (nx.b == b + 1) {
        if ((r = collect_sync(nx)) < 0) return r;
        nx.redo = false;
      }
    }
    return deliver(o);
  };
  auto cleanup = [&]() {
    for (Out& o : ot)
      if (o.th.joinable()) o.th.join();
  };
  const int fstep = input_planes(c->P) == 4 ? FFV1HIP_PLANES_YUVA : FFV1HIP_PLANES;  // plane pointers per frame
  for (int j = 0, base = 0; base < n_frames; j++, base += c->max_batch) {
    const int n = std::min(c->max_batch, n_frames - base);
    const int set = j % P.nsets;
    // batch j's packets go where batch j - 2's were, and with two frame sets
    // its frames too: batch j - 2 is collected before they are staged; with
    // three, before batch j launches (its frames and batch j - 1's stay in
    // place for a budget re-encode)
    if (P.nsets == 2 && (rc = retire(c->nsub - 2)) < 0) break;
    for (int i = 0; i < n && rc >= 0; i++)
      rc = stage_frame(c, set, i, planes + fstep * (base + i), strides + fstep * (base + i));
    if (rc >= 0 && P.nsets == 3) rc = retire(c->nsub - 2);
    if (rc >= 0) rc = launch_staged(c, set, n);
    if (rc < 0) break;
    Out& o = ot[(c->nsub - 1) & 1];
    if (P.overlap) {
      collect_async(o, c->nsub - 1, base);
    } else {
      o.b = c->nsub - 1;
      o.base = base;
      o.n = n;
      if ((rc = collect_sync(o)) < 0 || (rc = deliver(o)) < 0) break;
    }
  }
  if (rc >= 0 && P.overlap) {
    if ((rc = retire(c->nsub - 2)) >= 0) rc = retire(c->nsub - 1);
  }
  cleanup();
  if (P.dbg)
    std::fprintf(stderr, "hostdbg: %d frames, %d copy threads: slot wait %.3f s, copy in %.3f s, DMA issue %.3f s, "
                         "collector join wait %.3f s, batch wait (collectors) %.3f s; collectors: D2H %.3f s (sizes %.3f, "
                         "copy %.3f), into the buffer %.3f s\n",
                 n_frames, P.pool->size(), P.t_slot, P.t_copy, P.t_dma, P.t_join, P.t_settle, P.t_d2h, P.t_sizes,
                 P.t_dcopy, P.t_out);
  return rc;
}

int ffv1hip_encode2_delay(ffv1hip_ctx* c) {
  if (!c) return set_err(-22, "null ctx");
  HIP_TRY(hipSetDevice(c->device));
  const int rc = pipe_open(c);
  if (rc < 0) return rc;
  return (c->pipe.overlap ? 2 : 1) * c->max_batch - 1;
}

// The oldest launched batch's packets become the ones handed out.
static int collect_ready(ffv1hip_ctx* c) {
  ffv1hip_ctx::Launched l = c->launched.front();
  c->launched.pop_front();
  ffv1hip_ctx::Ready& R = c->ready;
  const uint8_t* h = nullptr;
  const int rc = collect(c, l.b, R.size, R.off, &h);
  if (rc < 0) return rc;
  R.base = h;
  R.key = c->hist[l.b & 1].keys;
  R.pts = std::move(l.pts);
  R.next = 0;
  return 0;
}

int ffv1hip_encode2(ffv1hip_ctx* c, const void* const planes[4], const int strides[4], int64_t pts,
                    uint8_t* out, int64_t out_cap, int64_t* size, int64_t* pts_out, int* key, int* got_packet) {
  if (!c || !got_packet) return set_err(-22, "null argument");
  *got_packet = 0;
  HIP_TRY(hipSetDevice(c->device));
  int rc = pipe_open(c);
  if (rc < 0) return rc;
  ffv1hip_ctx::Ready& R = c->ready;
  // with two frame sets a batch codes while the next one queues: batches are
  // collected once two are in flight (the encoder's delay is two batches)
  const size_t inflight = c->pipe.overlap ? 2 : 1;
  const bool drained = R.next >= R.size.size();
  if (planes) {
    if (!strides) return set_err(-22, "null strides");
    if (int64_t(c->q_pts.size()) >= c->max_batch)
      return set_err(-11, "frame queue full (%d frames): drain the packets first", c->max_batch);
    // the set this frame goes to must not hold a launched batch's frames
    // (a budget re-encode reads them): that batch is collected first
    if (c->q_pts.empty() && c->launched.size() >= inflight) {
      if (!drained) return set_err(-11, "packets pending: drain them first");
      if ((rc = collect_ready(c)) < 0) return rc;
    }
    // the frame is copied into the next batch slot (the caller keeps
    // ownership: it may reuse the buffer once the call returns)
    if ((rc = stage_frame(c, c->q_set, int64_t(c->q_pts.size()), planes, strides)) < 0) return rc;
    if (c->direct_pending) {  // straight from the caller's pinned memory: done before the call returns
      if (!c->direct_ev) HIP_TRY(hipEventCreateWithFlags(&c->direct_ev, hipEventDisableTiming));
      HIP_TRY(hipEventRecord(c->direct_ev, c->pipe.xfer));
      HIP_TRY(hipEventSynchronize(c->direct_ev));
      c->direct_pending = false;
    }
    c->q_pts.push_back(pts);
    if (int(c->q_pts.size()) == c->max_batch) {
      if ((rc = launch_staged(c, c->q_set, c->max_batch)) < 0) return rc;
      c->launched.push_back(ffv1hip_ctx::Launched{c->nsub - 1, std::move(c->q_pts)});
      c->q_pts.clear();
      if (c->pipe.overlap) c->q_set ^= 1;
    }
    if (R.next >= R.size.size() && c->launched.size() >= inflight && (rc = collect_ready(c)) < 0) return rc;
  } else if (R.next >= R.size.size()) {  // flush: what is launched, then what is queued
    if (c->launched.empty() && !c->q_pts.empty()) {
      if ((rc = launch_staged(c, c->q_set, int(c->q_pts.size()))) < 0) return rc;
      c->launched.push_back(ffv1hip_ctx::Launched{c->nsub - 1, std::move(c->q_pts)});
      c->q_pts.clear();
      if (c->pipe.overlap) c->q_set ^= 1;
    }
    if (!c->launched.empty() && (rc = collect_ready(c)) < 0) return rc;
  }
  c->last_out = -1;
  if (R.next >= R.size.size()) return 0;
  const size_t i = R.next;
  if (out) {
    // a slice budget re-encode can make packets larger than the
    // ffv1hip_max_packet_size the buffer was sized for: the frame is taken,
    // the packet waits for a call with a larger buffer
    if (R.size[i] > out_cap) {
      if (size) *size = R.size[i];
      return set_err(-28, "packet of %lld bytes, buffer %lld", (long long)R.size[i], (long long)out_cap);
    }
    pool_copy2d(*c->pipe.pool_out, out, R.size[i], R.base + R.off[i], R.size[i], R.size[i], 1);
  }
  if (size) *size = R.size[i];
  if (pts_out) *pts_out = R.pts[i];
  if (key) *key = R.key[i];
  *got_packet = 1;
  c->last_out = int64_t(i);
  R.next++;
  return 0;
}

int64_t ffv1hip_encode2_last_packet(ffv1hip_ctx* c, uint8_t* out, int64_t cap) {
  if (!c) return set_err(-22, "null ctx");
  const ffv1hip_ctx::Ready& R = c->ready;
  if (c->last_out < 0 || size_t(c->last_out) >= R.size.size()) return set_err(-22, "no packet handed out");
  const size_t i = size_t(c->last_out);
  if (R.size[i] > cap) return set_err(-28, "packet of %lld bytes, buffer %lld", (long long)R.size[i], (long long)cap);
  if (R.size[i] && !out) return set_err(-22, "null buffer");
  if (R.size[i]) pool_copy2d(*c->pipe.pool_out, out, R.size[i], R.base + R.off[i], R.size[i], R.size[i], 1);
  return R.size[i];
}

int ffv1hip_host_register(ffv1hip_ctx* c, void* ptr, int64_t bytes) {
  if (!c || !ptr || bytes <= 0) return set_err(-22, "null or empty range");
  const uintptr_t a = reinterpret_cast<uintptr_t>(ptr);
  auto it = c->host_ranges.lower_bound(a);
  if ((it != c->host_ranges.end() && it->first < a + uintptr_t(bytes)) ||
      (it != c->host_ranges.begin() && std::prev(it)->first + uintptr_t(std::prev(it)->second.bytes) > a))
    return set_err(-22, "the range overlaps a registered one");
  HIP_TRY(hipSetDevice(c->device));
  bool owned = true;
  const hipError_t e = hipHostRegister(ptr, size_t(bytes), hipHostRegisterDefault);
  if (e == hipErrorHostMemoryAlreadyRegistered) {
    owned = false;  // pinned by the process itself: left so on unregister
  } else if (e != hipSuccess) {
    (void)hipGetLastError();
    return set_err(-12, "hipHostRegister of %lld bytes: %s", (long long)bytes, hipGetErrorString(e));
  }
  (void)hipGetLastError();
  c->host_ranges[a] = ffv1hip_ctx::HostRange{bytes, owned};
  return 0;
}

int ffv1hip_host_unregister(ffv1hip_ctx* c, void* ptr) {
  if (!c) return set_err(-22, "null ctx");
  auto it = c->host_ranges.find(reinterpret_cast<uintptr_t>(ptr));
  if (it == c->host_ranges.end()) return set_err(-22, "no range registered at %p", ptr);
  HIP_TRY(hipSetDevice(c->device));
  if (c->pipe.xfer) HIP_TRY(hipStreamSynchronize(c->pipe.xfer));  // no copy from it is in flight
  if (it->second.owned) HIP_TRY(hipHostUnregister(ptr));
  c->host_ranges.erase(it);
  return 0;
}

int ffv1hip_set_profiling(ffv1hip_ctx* c, int enable) {
  if (!c) return set_err(-22, "null ctx");
  HIP_TRY(hipSetDevice(c->device));
  for (hipEvent_t& e : c->ev)
    if (!e) HIP_TRY(hipEventCreate(&e));
  c->profiling = enable != 0;
  c->nkev = 0;  // kernel stats accumulate from here
  return 0;
}

int ffv1hip_last_kernel_ms(ffv1hip_ctx* c, float* encode_ms, float* assemble_ms) {
  if (!c || !c->profiling) return set_err(-22, "profiling not enabled");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipEventSynchronize(c->ev[2]));
  float a = 0.f, b = 0.f;
  HIP_TRY(hipEventElapsedTime(&a, c->ev[0], c->ev[1]));
  HIP_TRY(hipEventElapsedTime(&b, c->ev[1], c->ev[2]));
  if (encode_ms) *encode_ms = a;
  if (assemble_ms) *assemble_ms = b;
  return 0;
}

int ffv1hip_last_kernel_stats(ffv1hip_ctx* c, ffv1hip_kernel_stats* out) {
  if (!c || !out || !c->profiling) return set_err(-22, "profiling not enabled");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipEventSynchronize(c->ev[2]));
  ffv1hip_kernel_stats s{};
  for (int j = 0; j < c->nkev; j++) {
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, c->kev[2 * j], c->kev[2 * j + 1]));
    switch (c->kev_kind[j]) {
      case 0: s.symbols_ms += ms; s.symbols_launches++; break;
      case 1: s.code_ms += ms; s.code_launches++; break;
      case 2: s.states_ms += ms; s.states_launches++; break;
      case 4: s.layout_ms += ms; s.layout_launches++; break;
      case 5: s.bits_ms += ms; s.bits_launches++; break;
      case 6: s.sink_ms += ms; s.sink_launches++; break;
      case 7: s.dseg_ms += ms; s.dseg_launches++; break;
      case 8: s.dfix_ms += ms; s.dfix_launches++; break;
      default: s.assemble_ms += ms; s.assemble_launches++; break;
    }
  }
  s.frames_coded_per_launch_max = c->last_nsegs;
  *out = s;
  return 0;
}

int64_t ffv1hip_get_slice_states(ffv1hip_ctx* c, uint8_t* buf, int64_t cap) {
  if (!c) return set_err(-22, "null ctx");
  const int64_t n = int64_t(c->pcount) * c->contexts * 32 * c->nslices;
  if (!buf) return n;
  if (cap < n) return set_err(-22, "buffer too small");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(buf, c->d_persist[c->pcur], n, hipMemcpyDeviceToHost));
  return n;
}

int ffv1hip_set_picture_number(ffv1hip_ctx* c, int64_t picture_number) {
  if (!c || picture_number < 0) return set_err(-22, "invalid arguments");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipDeviceSynchronize());
  c->picture_number = picture_number;
  return 0;
}

int ffv1hip_set_slice_states(ffv1hip_ctx* c, const uint8_t* buf, int64_t size) {
  if (!c || !buf) return set_err(-22, "null argument");
  const int64_t n = int64_t(c->pcount) * c->contexts * 32 * c->nslices;
  if (size != n) return set_err(-22, "state blob is %lld bytes, expected %lld", (long long)size, (long long)n);
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(c->d_persist[c->pcur], buf, n, hipMemcpyHostToDevice));
  c->have_states = true;
  return 0;
}

int64_t ffv1hip_get_slice_states_device(ffv1hip_ctx* c, void* d_buf, int64_t cap, void* stream) {
  if (!c) return set_err(-22, "null ctx");
  const int64_t n = int64_t(c->pcount) * c->contexts * 32 * c->nslices;
  if (!d_buf) return n;
  if (cap < n) return set_err(-22, "buffer too small");
  HIP_TRY(hipSetDevice(c->device));
  // the carry is complete once the batch is settled (a slice over the
  // budget re-encodes it); the copy then waits for the batch on the device
  const int rc = settle_batch(c, c->nsub - 1);
  if (rc < 0) return rc;
  hipStream_t const s = stream ? reinterpret_cast<hipStream_t>(stream) : c->stream;
  if (c->dep_valid) HIP_TRY(hipStreamWaitEvent(s, c->done_ev, 0));
  HIP_TRY(hipMemcpyAsync(d_buf, c->d_persist[c->pcur], size_t(n), hipMemcpyDeviceToDevice, s));
  if (s != c->stream) {
    // the context's next batches rewrite d_persist[pcur] (two batches on):
    // they start after this read on the caller's stream
    if (!c->xchg_ev) HIP_TRY(hipEventCreateWithFlags(&c->xchg_ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(c->xchg_ev, s));
    HIP_TRY(hipStreamWaitEvent(c->stream, c->xchg_ev, 0));
    HIP_TRY(hipEventRecord(c->dep_ev, c->stream));
    c->dep_valid = true;
  }
  return n;
}

int ffv1hip_set_slice_states_device(ffv1hip_ctx* c, const void* d_buf, int64_t size, void* stream) {
  if (!c || !d_buf) return set_err(-22, "null argument");
  const int64_t n = int64_t(c->pcount) * c->contexts * 32 * c->nslices;
  if (size != n) return set_err(-22, "state blob is %lld bytes, expected %lld", (long long)size, (long long)n);
  HIP_TRY(hipSetDevice(c->device));
  if (stream) {  // what the caller queued (the receive) first
    if (!c->xchg_ev) HIP_TRY(hipEventCreateWithFlags(&c->xchg_ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(c->xchg_ev, reinterpret_cast<hipStream_t>(stream)));
    HIP_TRY(hipStreamWaitEvent(c->stream, c->xchg_ev, 0));
  }
  if (c->dep_valid) HIP_TRY(hipStreamWaitEvent(c->stream, c->done_ev, 0));  // the last batch is done with the carry
  HIP_TRY(hipMemcpyAsync(c->d_persist[c->pcur], d_buf, size_t(n), hipMemcpyDeviceToDevice, c->stream));
  // the next batch (its walk or chained coder, and its coder stream) starts after the copy
  HIP_TRY(hipEventRecord(c->dep_ev, c->stream));
  HIP_TRY(hipEventRecord(c->done_ev, c->stream));
  c->dep_valid = true;
  c->have_states = true;
  // ... and so does the caller's stream: d_buf may be reused on it once the
  // copy has read it (include/ffv1hip.h)
  if (stream) HIP_TRY(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), c->done_ev, 0));
  return 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Decoder: the FFV1 decoder's AVCodec callbacks (ffv1dec.c decode_init :1007,
// decode_frame :896-1005, decode_end) for the streams this library encodes
// (version 3, range coder, context model 0).  Host work is the reference
// decoder's own host work: the key bit and the slice chain read backwards
// from the packet end (ffv1dec.c:931-989); the slices decode on the GPU.
struct ffv1hip_dec {
  Knobs knobs;
  int pcount = 2;  // plane contexts: 2, 3 with alpha
  ffv1hip_params P{};
  int device = 0;
  int nslices = 0;
  int contexts = 0;
  int64_t state_bytes = 0;
  int64_t frame_bytes = 0;
  int64_t plane_off[kMaxPlanes]{};
  int plane_w[kMaxPlanes]{};  // samples per row (bgr0 / RGB32: 4-byte pixels; YA8: 2-byte Y, A pairs)
  int out_planes = 0;      // planes handed back per frame (bgr0, RGB32, YA8: one packed plane)
  int out_rows[kMaxPlanes]{};
  int in_stride = 3;       // plane pointers per frame in ffv1hip_decode's arrays (4 for YUVA)
  int row_cap = 0;
  bool global_states = false;
  bool swap = false;  // range coder, YCbCr: one plane group's states in the LDS at a time
  bool have_states = false;
  bool have_last = false;  // d_last holds the previous picture (concealment)
  std::vector<SliceGeom> geom;
  uint8_t* d_persist[2] = {nullptr, nullptr};  // read [pcur], written [pcur ^ 1]
  int pcur = 0;
  SliceGeom* d_geom = nullptr;
  int16_t* d_qt = nullptr;
  uint8_t* d_tabs = nullptr;  // frame table to0 | to1, default table to0 | to1
  int32_t* d_stab = nullptr;  // the same frame table as pairs and the quant tables, int32 (DecodeArgs::stab)
  int* d_status = nullptr;
  uint8_t* d_sticky = nullptr;  // [slice] slice_damaged across calls
  uint8_t* d_last = nullptr;
  uint8_t* d_init = nullptr;  // initial states from the extradata (2-pass streams)
  hipStream_t stream = nullptr;
  int last_damaged = 0;
};

static void dec_free(ffv1hip_dec* d) {
  (void)hipFree(d->d_persist[0]);
  (void)hipFree(d->d_persist[1]);
  (void)hipFree(d->d_geom);
  (void)hipFree(d->d_qt);
  (void)hipFree(d->d_tabs);
  (void)hipFree(d->d_stab);
  (void)hipFree(d->d_status);
  (void)hipFree(d->d_sticky);
  (void)hipFree(d->d_last);
  if (d->d_init) (void)hipFree(d->d_init);
  if (d->stream) (void)hipStreamDestroy(d->stream);
}

// Range decoder over host bytes (rangecoder.h:104-147), for the extradata.
struct HostRacDec {
  const uint8_t* b;
  size_t n, pos = 2;
  int low, range = 0xFF00;
  const Tables* t;
  HostRacDec(const uint8_t* buf, size_t size, const Tables* tab) : b(buf), n(size), low((buf[0] << 8) | buf[1]), t(tab) {}
  int get(uint8_t* st) {
    const int r1 = (range * *st) >> 8;
    int bit;
    range -= r1;
    if (low < range) {
      bit = 0;
      *st = t->to0[*st];
    } else {
      low -= range;
      range = r1;
      bit = 1;
      *st = t->to1[*st];
    }
    if (range < 0x100) {
      range <<= 8;
      low <<= 8;
      if (pos < n) low += b[pos];
      pos++;
    }
    return bit;
  }
  int symbol(uint8_t* st, bool sgn) {
    if (get(st)) return 0;
    int e = 0;
    while (get(st + 1 + std::min(e, 9)))
      if (++e > 31) return 0;
    unsigned a = 1;
    for (int i = e - 1; i >= 0; i--) a = 2 * a + unsigned(get(st + 22 + std::min(i, 9)));
    return sgn && get(st + 11 + std::min(e, 10)) ? -int(a) : int(a);
  }
};

// read_extra_header (ffv1dec.c:509-631) as far as the custom transition
// table and the initial states, into c->frame / c->init_states; the
// caller compares the whole extradata afterwards.
static void read_extra_states(const uint8_t* ex, int size, ffv1hip_ctx* c) {
  if (size < 2) return;
  HostRacDec r(ex, size_t(size), &c->dflt);
  uint8_t st[32];
  std::memset(st, 128, 32);
  const int version = r.symbol(st, false);
  if (version > 2) (void)r.symbol(st, false);  // micro_version
  const int ac = r.symbol(st, false);
  if (ac == 2) {
    uint8_t stt[256] = {0};
    for (int i = 1; i < 256; i++) stt[i] = uint8_t(r.symbol(st, true) + c->dflt.to1[i]);
    c->frame = c->dflt;
    for (int i = 1; i < 256; i++) {
      c->frame.to1[i] = stt[i];
      c->frame.to0[256 - i] = uint8_t(256 - stt[i]);
    }
  }
  (void)r.symbol(st, false);  // colorspace
  (void)r.symbol(st, false);  // bits_per_raw_sample
  (void)r.get(st);            // chroma_planes
  (void)r.symbol(st, false);  // chroma_h_shift
  (void)r.symbol(st, false);  // chroma_v_shift
  (void)r.get(st);            // transparency
  (void)r.symbol(st, false);  // num_h_slices - 1
  (void)r.symbol(st, false);  // num_v_slices - 1
  const int nq = r.symbol(st, false);
  if (nq < 1 || nq > 2) return;
  for (int i = 0; i < nq; i++)  // the quant tables (ffv1dec.c:475-507), skipped
    for (int t = 0; t < 5; t++) {
      uint8_t qs[32];
      std::memset(qs, 128, 32);
      for (int k = 0; k < 128;) {
        const unsigned len = unsigned(r.symbol(qs, false)) + 1u;
        if (len > unsigned(128 - k) || !len) return;
        k += int(len);
      }
    }
  // The initial states come in the encoder's context numbering and count
  // (666 / 7563, ffv1enc.c:868-869), which is what the encoder wrote.  The
  // reference decoder counts contexts from the tables it read instead
  // (ffv1dec.c:497-507), which above 8 bits (9-level tables: 365 / 4105
  // contexts) is fewer than the encoder wrote, so it misreads a 2-pass
  // extradata there; this decoder reads what was written.
  const int counts[2] = {contexts_of(0), contexts_of(1)};
  uint8_t st2[32][32];
  std::memset(st2, 128, sizeof(st2));
  for (int i = 0; i < nq; i++) {  // ffv1dec.c:592-601
    if (!r.get(st)) continue;
    std::vector<uint8_t>& is = c->init_states[i];
    is.assign(size_t(counts[i]) * 32, 128);
    for (size_t j = 0; j < is.size(); j++) {
      const int pred = j >= 32 ? is[j - 32] : 128;
      is[j] = uint8_t((pred + r.symbol(st2[j & 31], true)) & 0xFF);
    }
  }
}

// The context states a slice starts from (ff_ffv1_clear_slice_state): all
// 128 for the range coder, VlcState{drift 0, error_sum 4, bias 0, count 1}
// per context for Golomb-Rice.
static int dec_reset_states(ffv1hip_dec* d) {
  for (uint8_t* pb : d->d_persist) {
    if (d->P.ac) {
      HIP_TRY(hipMemset(pb, 128, size_t(d->state_bytes) * d->nslices));
    } else {
      std::vector<uint64_t> v(size_t(d->state_bytes / 8) * d->nslices, uint64_t(4) << 16 | uint64_t(1) << 40);
      HIP_TRY(hipMemcpy(pb, v.data(), v.size() * 8, hipMemcpyHostToDevice));
    }
  }
  HIP_TRY(hipMemset(d->d_sticky, 0, size_t(d->nslices)));
  return 0;
}

extern "C" {

ffv1hip_dec* ffv1hip_dec_create(const ffv1hip_params* params, const uint8_t* extradata, int extradata_size,
                                int device, int* err) {
  auto fail = [&](int code) -> ffv1hip_dec* {
    if (err) *err = code;
    return nullptr;
  };
  if (!params) return fail(set_err(-22, "invalid arguments"));
  const ffv1hip_params& p = *params;
  if ((p.version == 2 && p.ec) || p.version > 4 || p.num_h_slices * p.num_v_slices > 256 || p.bits_per_raw_sample < 8 ||
      p.bits_per_raw_sample > 16 || p.width <= 0 || p.height <= 0 || p.num_h_slices <= 0 || p.num_v_slices <= 0 ||
      (p.version < 2 && p.num_h_slices * p.num_v_slices != 1) || p.context_model < 0 || p.context_model > 1 ||
      p.colorspace < 0 || p.colorspace > 1 || p.ac < 0 || p.ac > 2)
    return fail(set_err(-38, "GPU decoder: unsupported parameter set"));
  if (p.version > 4)
    return fail(set_err(-38, "GPU decoder: unsupported parameter set"));
  // The stream's extradata must be the one these parameters produce
  // (read_extradata, ffv1dec.c:509-631, would derive the same parameters);
  // versions 0 and 1 have none, their header is in band.
  ffv1hip_ctx tmp;
  tmp.P = p;
  tmp.contexts = contexts_of(p.context_model);
  tmp.dflt = default_tables();
  tmp.frame = p.ac == 2 ? custom_tables(tmp.dflt) : tmp.dflt;
  quant_set(tmp.qt, p.context_model, p.bits_per_raw_sample);
  // a 2-pass stream carries its own (sorted) custom table and initial
  // states: take them from the extradata, the rest must be what p produces
  if (p.version >= 2 && extradata && extradata_size > 4 && p.ac)
    read_extra_states(extradata, extradata_size - 4, &tmp);
  build_extradata(&tmp);
  if (extradata_size != int(tmp.extradata.size()) ||
      (extradata_size && (!extradata || std::memcmp(extradata, tmp.extradata.data(), tmp.extradata.size()) != 0)))
    return fail(set_err(FFV1HIP_AVERROR_INVALIDDATA, "extradata does not match the parameters"));
  ffv1hip_dec* d = new ffv1hip_dec();
  if (parse_knobs(&d->knobs) < 0) {
    delete d;
    return fail(-22);
  }
  d->P = p;
  d->device = device;
  d->nslices = p.num_h_slices * p.num_v_slices;
  d->contexts = tmp.contexts;
  d->pcount = 2 + (p.transparency != 0);
  d->state_bytes = int64_t(d->pcount) * d->contexts * (p.ac ? 32 : 8);
  const int cw = p.chroma_planes ? -((-p.width) >> p.chroma_h_shift) : 0;
  const int ch = p.chroma_planes ? -((-p.height) >> p.chroma_v_shift) : 0;
  const bool bgr0 = p.sample_bytes == 4;
  const bool ya8 = is_ya8(p);
  // the encoder's input layout: Y, Cb, Cr, A (YUVA); YA8 one plane of Y, A
  // byte pairs; bgr0 / RGB32 one plane of 4-byte pixels
  const int64_t pb0 = int64_t(p.width) * p.height * p.sample_bytes * (ya8 ? 2 : 1);
  const int64_t pb1 = bgr0 ? 0 : int64_t(cw) * ch * p.sample_bytes;
  const bool yuva = p.transparency && !p.colorspace && p.chroma_planes;
  d->plane_off[0] = 0;
  d->plane_off[1] = pb0;
  d->plane_off[2] = pb0 + pb1;
  d->plane_off[3] = pb0 + 2 * pb1;
  d->plane_w[0] = p.width * (ya8 ? 2 : 1);
  d->plane_w[1] = d->plane_w[2] = cw;
  d->plane_w[3] = p.width;
  d->out_planes = bgr0 || ya8 ? 1 : p.chroma_planes ? 3 + (yuva ? 1 : 0) : 1;
  d->in_stride = yuva ? FFV1HIP_PLANES_YUVA : FFV1HIP_PLANES;
  d->out_rows[0] = d->out_rows[3] = p.height;
  d->out_rows[1] = d->out_rows[2] = ch;
  d->frame_bytes = (pb0 + 2 * pb1 + (yuva ? int64_t(p.width) * p.height * p.sample_bytes : 0) + 255) & ~int64_t(255);
  d->geom.resize(d->nslices);
  for (int s = 0; s < d->nslices; s++) {  // ffv1.c:117-145, ffv1dec.c:361-474
    SliceGeom& g = d->geom[s];
    std::memset(&g, 0, sizeof(g));
    const int sx = s % p.num_h_slices, sy = s / p.num_h_slices;
    const int x0 = int(int64_t(p.width) * sx / p.num_h_slices);
    const int y0 = int(int64_t(p.height) * sy / p.num_v_slices);
    g.px[0] = x0;
    g.py[0] = y0;
    g.pw[0] = int(int64_t(p.width) * (sx + 1) / p.num_h_slices) - x0;
    g.ph[0] = int(int64_t(p.height) * (sy + 1) / p.num_v_slices) - y0;
    for (int k = 1; k < 3; k++) {
      g.pw[k] = p.chroma_planes ? -((-g.pw[0]) >> p.chroma_h_shift) : 0;
      g.ph[k] = p.chroma_planes ? -((-g.ph[0]) >> p.chroma_v_shift) : 0;
      g.px[k] = x0 >> p.chroma_h_shift;
      g.py[k] = y0 >> p.chroma_v_shift;
    }
    if (yuva) {  // A at the luma rectangle
      g.px[3] = g.px[0]; g.py[3] = g.py[0]; g.pw[3] = g.pw[0]; g.ph[3] = g.ph[0];
    }
    d->row_cap = std::max(d->row_cap, g.pw[0]);
  }
  d->row_cap = (d->row_cap + 7) & ~7;
  // states in LDS when they fit beside the rows, else one global table per chain
  DecodeArgs la{};
  la.state_bytes = d->state_bytes;
  la.rgb = p.colorspace;
  la.transparency = p.transparency;
  la.row_cap = d->row_cap;
  la.context_model = p.context_model;
  constexpr int64_t kDecLds = 64 * 1024;
  d->global_states = decode_lds_bytes(la, false) > kDecLds;
  d->swap = !d->global_states && p.ac && !p.colorspace && p.chroma_planes && !p.transparency;
  if (decode_lds_bytes(la, true) > kDecLds) {
    delete d;
    return fail(set_err(-38, "GPU decoder: slice too wide for the LDS row buffer"));
  }
  auto init = [&]() -> int {
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
    HIP_TRY(hipMalloc(&d->d_persist[0], d->state_bytes * d->nslices));
    HIP_TRY(hipMalloc(&d->d_persist[1], d->state_bytes * d->nslices));
    HIP_TRY(hipMalloc(&d->d_geom, sizeof(SliceGeom) * d->nslices));
    HIP_TRY(hipMalloc(&d->d_qt, sizeof(int16_t) * 5 * 256));
    HIP_TRY(hipMalloc(&d->d_tabs, 1024));
    HIP_TRY(hipMalloc(&d->d_status, sizeof(int) * 4));
    HIP_TRY(hipMalloc(&d->d_sticky, size_t(d->nslices)));
    HIP_TRY(hipMalloc(&d->d_last, size_t(d->frame_bytes)));
    HIP_TRY(hipMemcpy(d->d_geom, d->geom.data(), sizeof(SliceGeom) * d->nslices, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(d->d_qt, tmp.qt, sizeof(int16_t) * 5 * 256, hipMemcpyHostToDevice));
    uint8_t tabs[1024];
    std::memcpy(tabs, tmp.frame.to0, 256);
    std::memcpy(tabs + 256, tmp.frame.to1, 256);
    std::memcpy(tabs + 512, tmp.dflt.to0, 256);
    std::memcpy(tabs + 768, tmp.dflt.to1, 256);
    HIP_TRY(hipMemcpy(d->d_tabs, tabs, 1024, hipMemcpyHostToDevice));
    std::vector<int32_t> stab(256 + 5 * 256);
    for (int i = 0; i < 256; i++) stab[i] = int32_t(tmp.frame.to0[i]) | (int32_t(tmp.frame.to1[i]) << 8);
    for (int i = 0; i < 5 * 256; i++) stab[256 + i] = tmp.qt[i / 256][i % 256];
    HIP_TRY(hipMalloc(&d->d_stab, stab.size() * sizeof(int32_t)));
    HIP_TRY(hipMemcpy(d->d_stab, stab.data(), stab.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    const std::vector<uint8_t>& is = tmp.init_states[p.context_model];
    if (std::any_of(is.begin(), is.end(), [](uint8_t v) { return v != 128; })) {
      HIP_TRY(hipMalloc(&d->d_init, is.size()));
      HIP_TRY(hipMemcpy(d->d_init, is.data(), is.size(), hipMemcpyHostToDevice));
    }
    return dec_reset_states(d);
  };
  int rc = init();
  if (rc < 0) {
    dec_free(d);
    delete d;
    return fail(rc);
  }
  if (err) *err = 0;
  return d;
}

void ffv1hip_dec_destroy(ffv1hip_dec* d) {
  if (!d) return;
  (void)hipSetDevice(d->device);
  dec_free(d);
  delete d;
}

int ffv1hip_decode(ffv1hip_dec* d, const uint8_t* packets, const int64_t* sizes, int n_frames,
                   void* const* planes, const int* strides, int* key_flags) {
  if (!d || !packets || !sizes || n_frames < 0 || (n_frames && (!planes || !strides)))
    return set_err(-22, "null argument");
  d->last_damaged = 0;
  if (n_frames == 0) return 0;
  const ffv1hip_params& p = d->P;
  const int ns = d->nslices;
  const int trailer = 3 + (p.ec ? 5 : 0);
  std::vector<uint8_t> keys(n_frames);
  std::vector<int64_t> starts(size_t(n_frames) * ns), ends(size_t(n_frames) * ns);
  int64_t total = 0;
  for (int f = 0; f < n_frames; f++) {
    const uint8_t* pk = packets + total;
    const int64_t size = sizes[f];
    if (size < 2) return set_err(FFV1HIP_AVERROR_INVALIDDATA, "frame %d: packet too small", f);
    // key bit: the first decision with state 128 from range 0xFF00 (ffv1dec.c:931)
    keys[f] = ((pk[0] << 8) | pk[1]) >= 0x7F80;
    // the slice chain, from the packet end (ffv1dec.c:948-989); below v3
    // the only slice runs to the end
    const uint8_t* q = pk + size;
    for (int i = ns - 1; i >= 0; i--) {
      int64_t v;
      if (i || p.version > 2) {
        if (q - pk < trailer) return set_err(FFV1HIP_AVERROR_INVALIDDATA, "frame %d: slice %d trailer", f, i);
        v = ((int64_t(q[-trailer]) << 16) | (q[-trailer + 1] << 8) | q[-trailer + 2]) + trailer;
      } else {
        v = q - pk;
      }
      if (v > q - pk) return set_err(FFV1HIP_AVERROR_INVALIDDATA, "frame %d: slice %d size", f, i);
      ends[size_t(f) * ns + i] = (q - packets);
      q -= v;
      starts[size_t(f) * ns + i] = (q - packets);
    }
    if (q != pk) return set_err(FFV1HIP_AVERROR_INVALIDDATA, "frame %d: %d slices do not span the packet", f, ns);
    if (ends[size_t(f) * ns] - starts[size_t(f) * ns] < 2)
      return set_err(FFV1HIP_AVERROR_INVALIDDATA, "frame %d: first slice too small", f);
    total += size;
  }
  // slice CRCs (ffv1dec.c:963-977): a mismatch marks the slice damaged, it
  // is still decoded, then concealed; checked on host threads
  const size_t nse = size_t(n_frames) * ns;
  std::vector<uint8_t> damage(nse, 0);
  if (p.ec) {
    const int nt = int(std::max<size_t>(1, std::min<size_t>({nse, 16, std::thread::hardware_concurrency()})));
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; t++)
      pool.emplace_back([&, t] {
        for (size_t k = size_t(t); k < nse; k += size_t(nt))
          damage[k] = crc32_msb_fast(packets + starts[k], size_t(ends[k] - starts[k])) != 0;
      });
    for (auto& th : pool) th.join();
  }
  if (!keys[0] && !d->have_states)
    return set_err(FFV1HIP_AVERROR_INVALIDDATA, "stream does not start with a keyframe");
  std::vector<Segment> segs;
  for (int f = 0; f < n_frames; f++) {
    if (f == 0 || keys[f]) segs.push_back(Segment{f, 0, f == 0 && !keys[0], 0});
    segs.back().nframes++;
  }
  segs.back().save_states = 1;
  HIP_TRY(hipSetDevice(d->device));
  uint8_t* d_pk = nullptr;
  int64_t* d_se = nullptr;
  uint8_t* d_keys = nullptr;
  Segment* d_segs = nullptr;
  uint8_t* d_out = nullptr;
  uint8_t* d_dmg = nullptr;
  uint8_t* d_tables = nullptr;
  auto run = [&]() -> int {
    HIP_TRY(hipMalloc(&d_pk, size_t(total) + 64));
    HIP_TRY(hipMalloc(&d_se, 2 * nse * sizeof(int64_t)));
    HIP_TRY(hipMalloc(&d_keys, size_t(n_frames)));
    HIP_TRY(hipMalloc(&d_segs, segs.size() * sizeof(Segment)));
    HIP_TRY(hipMalloc(&d_out, size_t(d->frame_bytes) * n_frames));
    HIP_TRY(hipMalloc(&d_dmg, nse));
    if (d->global_states || d->swap) HIP_TRY(hipMalloc(&d_tables, size_t(d->state_bytes) * ns * segs.size()));
    HIP_TRY(hipMemsetAsync(d_pk + total, 0, 64, d->stream));
    // samples no slice codes (odd chroma offsets, ffv1enc.c:1186-1188) read as 0
    HIP_TRY(hipMemsetAsync(d_out, 0, size_t(d->frame_bytes) * n_frames, d->stream));
    HIP_TRY(hipMemcpyAsync(d_pk, packets, size_t(total), hipMemcpyHostToDevice, d->stream));
    HIP_TRY(hipMemcpyAsync(d_se, starts.data(), nse * sizeof(int64_t), hipMemcpyHostToDevice, d->stream));
    HIP_TRY(hipMemcpyAsync(d_se + nse, ends.data(), nse * sizeof(int64_t), hipMemcpyHostToDevice, d->stream));
    HIP_TRY(hipMemcpyAsync(d_keys, keys.data(), size_t(n_frames), hipMemcpyHostToDevice, d->stream));
    HIP_TRY(hipMemcpyAsync(d_segs, segs.data(), segs.size() * sizeof(Segment), hipMemcpyHostToDevice, d->stream));
    HIP_TRY(hipMemcpyAsync(d_dmg, damage.data(), nse, hipMemcpyHostToDevice, d->stream));
    HIP_TRY(hipMemsetAsync(d->d_status, 0, sizeof(int) * 4, d->stream));
    DecodeArgs a{};
    a.pkts = d_pk;
    a.slice_start = d_se;
    a.slice_end = d_se + nse;
    a.keyflags = d_keys;
    a.segs = d_segs;
    a.geom = d->d_geom;
    a.nslices = ns;
    a.nplanes = p.chroma_planes ? 3 + (p.transparency && !p.colorspace ? 1 : 0) : 1;
    a.transparency = p.transparency;
    a.ya8 = is_ya8(p);
    a.pcount = d->pcount;
    a.qt = d->d_qt;
    a.ftab = d->d_tabs;
    a.dtab = d->d_tabs + 512;
    a.stab = d->d_stab;
    a.state_bytes = d->state_bytes;
    a.persist_in = d->d_persist[d->pcur];
    a.persist_out = d->d_persist[d->pcur ^ 1];
    a.tables = d_tables;
    a.out = d_out;
    a.frame_bytes = d->frame_bytes;
    for (int k = 0; k < kMaxPlanes; k++) {
      a.plane_off[k] = d->plane_off[k];
      a.plane_w[k] = d->plane_w[k];
    }
    a.sample_bytes = p.sample_bytes;
    a.packed_at_lsb = p.packed_at_lsb;
    a.msb_shift = 16 - p.bits_per_raw_sample;
    a.coded_bits = coded_bits(p);
    a.width = p.width;
    a.height = p.height;
    a.num_h = p.num_h_slices;
    a.num_v = p.num_v_slices;
    a.context_model = p.context_model;
    a.version = p.version;
    a.ac = p.ac;
    a.ec = p.ec;
    a.rgb = p.colorspace;
    a.rct_offset = 1 << p.bits_per_raw_sample;
    a.contexts = d->contexts;
    a.chroma_planes = p.chroma_planes;
    a.chroma_h_shift = p.chroma_h_shift;
    a.chroma_v_shift = p.chroma_v_shift;
    a.bits_per_raw_sample = p.bits_per_raw_sample;
    a.row_cap = d->row_cap;
    a.status = d->d_status;
    a.damage = d_dmg;
    a.last = d->have_last ? d->d_last : nullptr;
    a.sticky = d->d_sticky;
    a.nframes = n_frames;
    a.init = d->d_init;
    a.swap = d->swap;
    if (launch_decode(a, int(segs.size()), d->stream) < 0)
      return set_err(-5, "ffv1_decode_slices launch failed: %s", hipGetErrorString(hipGetLastError()));
    int status = 0;
    HIP_TRY(hipMemcpyAsync(&status, d->d_status, sizeof(int), hipMemcpyDeviceToHost, d->stream));
    HIP_TRY(hipStreamSynchronize(d->stream));
    if (status) return set_err(FFV1HIP_AVERROR_INVALIDDATA, "%d frame(s) with a bad key bit or in-band header", status);
    if (launch_conceal(a, d->stream) < 0)
      return set_err(-5, "ffv1_conceal launch failed: %s", hipGetErrorString(hipGetLastError()));
    HIP_TRY(hipMemcpyAsync(d->d_last, d_out + int64_t(n_frames - 1) * d->frame_bytes, size_t(d->frame_bytes),
                           hipMemcpyDeviceToDevice, d->stream));
    HIP_TRY(hipMemcpyAsync(damage.data(), d_dmg, nse, hipMemcpyDeviceToHost, d->stream));
    for (int f = 0; f < n_frames; f++)
      for (int k = 0; k < d->out_planes; k++) {
        const int64_t wb = int64_t(d->plane_w[k]) * p.sample_bytes;
        HIP_TRY(hipMemcpy2DAsync(planes[d->in_stride * f + k], strides[d->in_stride * f + k],
                                 d_out + int64_t(f) * d->frame_bytes + d->plane_off[k], size_t(wb), size_t(wb),
                                 d->out_rows[k], hipMemcpyDeviceToHost, d->stream));
      }
    HIP_TRY(hipStreamSynchronize(d->stream));
    for (uint8_t v : damage) d->last_damaged += v != 0;
    return 0;
  };
  int rc = run();
  (void)hipFree(d_pk);
  (void)hipFree(d_se);
  (void)hipFree(d_keys);
  (void)hipFree(d_segs);
  (void)hipFree(d_out);
  (void)hipFree(d_dmg);
  if (d_tables) (void)hipFree(d_tables);
  if (rc < 0) return rc;
  d->pcur ^= 1;
  d->have_states = true;
  d->have_last = true;
  if (key_flags)
    for (int f = 0; f < n_frames; f++) key_flags[f] = keys[f];
  return 0;
}

int ffv1hip_dec_damaged_slices(const ffv1hip_dec* d) { return d ? d->last_damaged : -22; }

void ffv1hip_dec_reset(ffv1hip_dec* d) {
  if (!d) return;
  d->have_states = false;
  d->have_last = false;
  (void)hipSetDevice(d->device);
  (void)dec_reset_states(d);
}

}  // extern "C"
