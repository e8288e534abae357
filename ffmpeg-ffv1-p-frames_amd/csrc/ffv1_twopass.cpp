// ffv1_twopass.cpp -- the 2-pass mode of encode_init (ffv1enc.c:898-986):
// pass 1 counts, per adaptive state value and per (context, slot), how many
// zero and one decisions the plane symbols coded (put_symbol_inline's
// statistics, :190-199, written into stats_out by encode_frame at the end
// of the stream, :1236-1277); pass 2 reads that text back, re-orders the
// custom transition table by the counts (sort_stt, :621-667) and derives
// every context's initial states (find_best_state, :139-183).  The counting
// runs on the GPU (ffv1_kernels.hip, ffv1_stats_*); this file is the
// init-time host arithmetic.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ffv1_internal.h"

namespace ffv1hip {

namespace {

// for a probability i/256 of a one after k decisions, the starting state
// whose adaptation through one_state codes them in the fewest bits
void find_best_state(uint8_t best[256][256], const uint8_t one_state[256]) {
  double l2[256] = {0};
  for (int i = 1; i < 256; i++) l2[i] = std::log2(i / 256.0);
  std::vector<double> occ(256), nocc(256);
  for (int i = 0; i < 256; i++) {
    double best_len[256];
    const double p = i / 256.0;
    for (double& b : best_len) b = double(1 << 30);
    const int j0 = i - 10 > 1 ? i - 10 : 1, j1 = i + 11 < 256 ? i + 11 : 256;
    for (int j = j0; j < j1; j++) {
      if (!one_state[j]) continue;
      std::fill(occ.begin(), occ.end(), 0.0);
      occ[j] = 1.0;
      double len = 0;
      for (int k = 0; k < 256; k++) {
        std::fill(nocc.begin(), nocc.end(), 0.0);
        for (int m = 1; m < 256; m++)
          if (occ[m]) len -= occ[m] * (p * l2[m] + (1 - p) * l2[256 - m]);
        if (len < best_len[k]) {
          best_len[k] = len;
          best[i][k] = uint8_t(j);
        }
        for (int m = 1; m < 256; m++)
          if (occ[m]) {
            nocc[one_state[m]] += occ[m] * p;
            nocc[256 - one_state[256 - m]] += occ[m] * (1 - p);
          }
        occ.swap(nocc);
      }
    }
  }
}

// The reference swaps the 64-bit counters through an int: FFSWAP(int, a, b)
// is { int tmp = b; b = a; a = tmp; } (libavutil/common.h:99), so b takes a
// whole and a takes b truncated to 32 bits and sign-extended.
void swap_through_int(uint64_t& a, uint64_t& b) {
  const int t = int(uint32_t(b));
  b = a;
  a = uint64_t(int64_t(t));
}

// COST(old, new) of the reference's macro, added term by term to s: the
// macros expand size0 / sizeX into one sum of eight products, evaluated left
// to right, and the swap test compares them to 1e-14, so the association
// matters
void add_cost(double& s, const uint64_t st[256][2], int o, int n) {
  s += double(st[o][0]) * -std::log2((256 - n) / 256.0);
  s += double(st[o][1]) * -std::log2(n / 256.0);
}

// COST2(i, a) + COST2(i2, b)
double cost_pair(const uint64_t st[256][2], int i, int a, int i2, int b) {
  double s = 0.0;
  add_cost(s, st, i, a);
  add_cost(s, st, 256 - i, 256 - a);
  add_cost(s, st, i2, b);
  add_cost(s, st, 256 - i2, 256 - b);
  return s;
}

void sort_stt(uint64_t st[256][2], uint8_t stt[256]) {
  bool changed;
  do {
    changed = false;
    for (int i = 12; i < 244; i++)
      for (int i2 = i + 1; i2 < 245 && i2 < i + 4; i2++) {
        const double size0 = cost_pair(st, i, i, i2, i2);
        const double sizeX = cost_pair(st, i, i2, i2, i);
        if (!(size0 - sizeX > size0 * (1e-14) && i != 128 && i2 != 128)) continue;
        std::swap(stt[i], stt[i2]);
        swap_through_int(st[i][0], st[i2][0]);
        swap_through_int(st[i][1], st[i2][1]);
        if (i != 256 - i2) {
          std::swap(stt[256 - i], stt[256 - i2]);
          swap_through_int(st[256 - i][0], st[256 - i2][0]);
          swap_through_int(st[256 - i][1], st[256 - i2][1]);
        }
        for (int j = 1; j < 256; j++) {
          if (stt[j] == i) stt[j] = uint8_t(i2);
          else if (stt[j] == i2) stt[j] = uint8_t(i);
          if (i != 256 - i2) {
            if (stt[256 - j] == 256 - i) stt[256 - j] = uint8_t(256 - i2);
            else if (stt[256 - j] == 256 - i2) stt[256 - j] = uint8_t(256 - i);
          }
        }
        changed = true;
      }
  } while (changed);
}

int clip(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }

}  // namespace

int pass2_states(const char* stats, bool custom, uint8_t stt[256], const uint8_t default_one[256],
                 std::vector<uint8_t> init[2], std::string* err) {
  const int counts[2] = {(11 * 11 * 11 + 1) / 2, (11 * 11 * 5 * 5 * 5 + 1) / 2};
  // per call (two contexts may initialise pass 2 at once)
  std::vector<uint64_t> rc_stat_v(256 * 2, 0);
  uint64_t(*rc_stat)[2] = reinterpret_cast<uint64_t(*)[2]>(rc_stat_v.data());
  std::vector<uint64_t> st2[2];
  for (int i = 0; i < 2; i++) st2[i].assign(size_t(counts[i]) * 64, 0);
  int gob_count = 0;
  const char* p = stats;
  char* next = nullptr;
  auto bad = [&](const char* what) {
    if (err) *err = std::string("2-pass statistics invalid at ") + what;
    return -1094995529;  // AVERROR_INVALIDDATA
  };
  for (;;) {  // every block in turn; the last one counts (ffv1enc.c:914-953)
    for (int j = 0; j < 256; j++)
      for (int i = 0; i < 2; i++) {
        rc_stat[j][i] = uint64_t(std::strtol(p, &next, 0));
        if (next == p) return bad("the state counts");
        p = next;
      }
    for (int i = 0; i < 2; i++)
      for (size_t j = 0; j < st2[i].size(); j++) {
        st2[i][j] = uint64_t(std::strtol(p, &next, 0));
        if (next == p) return bad("the context counts");
        p = next;
      }
    gob_count = int(std::strtol(p, &next, 0));
    if (next == p || gob_count <= 0) return bad("the keyframe count");
    p = next;
    while (*p == '\n' || *p == ' ') p++;
    if (!*p) break;
  }
  if (custom) sort_stt(rc_stat, stt);
  std::vector<uint8_t> best_v(256 * 256, 0);
  uint8_t(*best)[256] = reinterpret_cast<uint8_t(*)[256]>(best_v.data());
  find_best_state(best, custom ? stt : default_one);
  for (int i = 0; i < 2; i++) {
    std::vector<uint8_t>& is = init[i];
    is.assign(size_t(counts[i]) * 32, 128);
    for (int k = 0; k < 32; k++) {
      double a = 0, b = 0;
      int jp = 0;
      for (int j = 0; j < counts[i]; j++) {
        const uint64_t c0 = st2[i][(size_t(j) * 32 + k) * 2], c1 = st2[i][(size_t(j) * 32 + k) * 2 + 1];
        double pr = 128;
        if ((c0 + c1 > 200 && j) || a + b > 200) {
          if (a + b) pr = 256.0 * b / (a + b);
          is[size_t(jp) * 32 + k] = best[clip(int(std::round(pr)), 1, 255)][clip(int((a + b) / gob_count), 0, 255)];
          for (jp++; jp < j; jp++) is[size_t(jp) * 32 + k] = is[size_t(jp - 1) * 32 + k];
          a = b = 0;
        }
        a += double(c0);
        b += double(c1);
        if (a + b) pr = 256.0 * b / (a + b);
        is[size_t(j) * 32 + k] = best[clip(int(std::round(pr)), 1, 255)][clip(int((a + b) / gob_count), 0, 255)];
      }
    }
  }
  return 0;
}

std::string pass1_text(const uint64_t* rc_stat, const uint64_t* rc_stat2, int contexts, int model, int gob_count) {
  std::string out;
  char tmp[48];
  out.reserve(size_t(8231) * 64 * 3);
  for (int j = 0; j < 256; j++) {
    std::snprintf(tmp, sizeof(tmp), "%llu %llu ", (unsigned long long)rc_stat[2 * j],
                  (unsigned long long)rc_stat[2 * j + 1]);
    out += tmp;
  }
  out += "\n";
  const int counts[2] = {(11 * 11 * 11 + 1) / 2, (11 * 11 * 5 * 5 * 5 + 1) / 2};
  for (int i = 0; i < 2; i++)
    for (int j = 0; j < counts[i]; j++)
      for (int m = 0; m < 32; m++) {
        uint64_t a = 0, b = 0;
        if (i == model && j < contexts) {
          a = rc_stat2[(size_t(j) * 32 + m) * 2];
          b = rc_stat2[(size_t(j) * 32 + m) * 2 + 1];
        }
        std::snprintf(tmp, sizeof(tmp), "%llu %llu ", (unsigned long long)a, (unsigned long long)b);
        out += tmp;
      }
  std::snprintf(tmp, sizeof(tmp), "%d\n", gob_count);
  out += tmp;
  return out;
}

}  // namespace ffv1hip

// Host-only test hook (not part of include/ffv1hip.h): pass2_states on a
// stats_in text, for the sanitizer build's parser checks
// (tests/test_sanitize.py).  init0 / init1 receive 666 / 7563 x 32 states.
extern "C" int ffv1hip_internal_pass2_states(const char* stats, int custom, uint8_t* stt,
                                             const uint8_t* default_one, uint8_t* init0, uint8_t* init1) {
  std::vector<uint8_t> init[2];
  std::string err;
  const int rc = ffv1hip::pass2_states(stats, custom != 0, stt, default_one, init, &err);
  if (rc < 0) return rc;
  std::memcpy(init0, init[0].data(), init[0].size());
  std::memcpy(init1, init[1].data(), init[1].size());
  return 0;
}

// Host-only test hook (not part of include/ffv1hip.h): sort_stt on
// caller-given counts [256][2] and table, for the FFSWAP(int, ...)
// truncation check in tests/test_twopass_host.py.
extern "C" void ffv1hip_internal_sort_stt(uint64_t* rc_stat, uint8_t* stt) {
  ffv1hip::sort_stt(reinterpret_cast<uint64_t(*)[2]>(rc_stat), stt);
}
