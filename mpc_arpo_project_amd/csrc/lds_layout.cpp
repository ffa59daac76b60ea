// lds_layout.cpp -- LDS bank-conflict model and optimiser of the solve steps (symbolic.hpp).
//
// The solve steps are LDS-bound: with four waves per CU the LDS array is the shared resource
// (occupancy scan: 1 -> 4 instances per CU gives only 2.9x; removing the conflict-aware matrix
// layout costs 34 % of the kernel time).  A step is 16 ds_read_b64 (8 matrix operands, 8 vector
// operands) and 4 ds_add_f64 per lane; its LDS time grows with the bank conflicts of each
// instruction (MI355X_MICROARCH.md, LDS): a ds_read_b64 serves two 32-lane halves, one cycle per
// distinct address on the busiest bank (slot mod 32, equal addresses broadcast); a ds_add_f64 or
// ds_write_b64 serves four 16-lane groups, one cycle per lane on the busiest bank (slot mod 16,
// equal addresses serialise).
//
// optimize_lds() minimises the modelled cycles of the solve steps plus the per-iteration vector
// passes (right-hand side scatter, solution gather) by simulated annealing over
//   * per step: the position (lane, instruction) of every segment, the operand order of every
//     term (a b = b a exactly), the term order of a segment and the pairing of the terms of one
//     target into segments (these two change the rounding of the target's sum only);
//   * globally: the LDS slots of the solve-read matrix values (permutations inside the L-live
//     range and inside N | G | G') and of the vector entries (one permutation applied to the W,
//     C and 1/D regions together, so the slot-aligned vector passes stay aligned, restricted to
//     swaps that keep every L entry inside the L range the flat pass walks);
// and then gives every unused segment a sink in a free bank (adding -0.0 is an exact no-op, so any
// 1/D slot serves) and every padding term a zero slot of the least used bank (ZERO_BLOCK).  All
// slot changes are applied to every table of the plan (a relabelling of the LDS image).
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "symbolic.hpp"

namespace mpcqp {
namespace {

double envd(const char* k, double d) {
  const char* e = diag_env(k);
  return (e && *e) ? atof(e) : d;
}

constexpr int RBANKS = 32;  // ds_read_b64: double slot mod 32 per 32-lane half
constexpr int WBANKS = 16;  // ds_add_f64 / ds_write_b64: double slot mod 16 per 16-lane group

// distinct addresses on the busiest bank; `nz` zero-padding reads go to the zero slot of the
// least used bank (one cycle more there if it is not empty)
int read_cost(const int* a, int cnt, int nz) {
  int nb[RBANKS] = {};
  int seen[RBANKS][32];
  int mx = 0;
  for (int i = 0; i < cnt; ++i) {
    const int b = a[i] & (RBANKS - 1);
    bool dup = false;
    for (int k = 0; k < nb[b]; ++k)
      if (seen[b][k] == a[i]) {
        dup = true;
        break;
      }
    if (!dup) seen[b][nb[b]++] = a[i], mx = std::max(mx, nb[b]);
  }
  if (nz > 0) {
    int mn = nb[0];
    for (int b = 1; b < RBANKS; ++b) mn = std::min(mn, nb[b]);
    mx = std::max(mx, mn + 1);
  }
  return std::max(mx, 1);
}
// annealing objective: SM x the modelled cycles plus the number of excess addresses over all
// banks (a gradient on the plateaus of the max)
constexpr int SM = 8;
int read_cost_s(const int* a, int cnt, int nz) {
  int nb[RBANKS] = {};
  int seen[RBANKS][32];
  int mx = 0, ex = 0;
  for (int i = 0; i < cnt; ++i) {
    const int b = a[i] & (RBANKS - 1);
    bool dup = false;
    for (int k = 0; k < nb[b]; ++k)
      if (seen[b][k] == a[i]) {
        dup = true;
        break;
      }
    if (!dup) {
      if (nb[b]) ex++;
      seen[b][nb[b]++] = a[i], mx = std::max(mx, nb[b]);
    }
  }
  if (nz > 0) {
    int mn = nb[0];
    for (int b = 1; b < RBANKS; ++b) mn = std::min(mn, nb[b]);
    mx = std::max(mx, mn + 1);
  }
  return SM * std::max(mx, 1) + ex;
}
int write_cost_s(const int* a, int cnt) {
  int c[WBANKS] = {};
  int mx = 1, ex = 0;
  for (int i = 0; i < cnt; ++i) {
    const int k = ++c[a[i] & (WBANKS - 1)];
    if (k > 1) ex++;
    mx = std::max(mx, k);
  }
  return SM * mx + ex;
}
// lanes on the busiest bank (sinks of unused lanes go to free banks)
int write_cost(const int* a, int cnt) {
  int c[WBANKS] = {};
  int mx = 1;
  for (int i = 0; i < cnt; ++i) mx = std::max(mx, ++c[a[i] & (WBANKS - 1)]);
  return mx;
}

struct Seg {
  int a[2] = {-1, -1}, b[2] = {-1, -1};  // operand slots; -1: zero padding
  int t = -1;                            // target slot; -1: unused segment
};
typedef std::array<Seg, 256> Step;  // position q * 64 + lane

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 1) {}
  uint64_t next() {
    s ^= s >> 12, s ^= s << 25, s ^= s >> 27;
    return s * 0x2545F4914F6CDD1Dull;
  }
  int below(int n) { return (int)(next() % (uint64_t)n); }
  double unit() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
};

struct Opt {
  Plan& pl;
  std::vector<Step> st;       // forward steps, then backward steps
  std::vector<int> ren;       // slot -> slot (a permutation of the LDS image)
  explicit Opt(Plan& p) : pl(p) {}

  int phys(int x) const { return x < 0 ? -1 : ren[x]; }

  // ---- step-local group costs
  int rd_group(const Step& s, int c, int op, int h) const {
    int a[32], cnt = 0, nz = 0;
    const int q = c / 2, j = c % 2;
    for (int l = 32 * h; l < 32 * h + 32; ++l) {
      const Seg& g = s[q * 64 + l];
      const int x = op ? g.b[j] : g.a[j];
      if (x < 0)
        nz++;
      else
        a[cnt++] = ren[x];
    }
    return read_cost_s(a, cnt, nz);
  }
  int at_group(const Step& s, int q, int grp) const {
    if (q == 1 && pl.paired) return 0;  // segment 1 is summed into segment 0's atomic
    int a[16], cnt = 0;
    for (int l = 16 * grp; l < 16 * grp + 16; ++l) {
      const int t = s[q * 64 + l].t;
      if (t >= 0) a[cnt++] = ren[t];
    }
    return write_cost_s(a, cnt);
  }
  int step_cost(const Step& s) const {
    int c = 0;
    for (int k = 0; k < 8; ++k)
      for (int op = 0; op < 2; ++op)
        for (int h = 0; h < 2; ++h) c += rd_group(s, k, op, h);
    for (int q = 0; q < 4; ++q)
      for (int g = 0; g < 4; ++g) c += at_group(s, q, g);
    return c;
  }
  // vector passes: rhs scatter into C (ds_write_b64) and solution gather from W (ds_read_b64)
  int vec_cost() const {
    int c = 0;
    auto pass = [&](const std::vector<uint16_t>& ws, int slots) {
      for (int r = 0; r < slots; ++r) {
        int a[64];
        for (int l = 0; l < 64; ++l) a[l] = ws[64 * r + l] - pl.W;  // vector index
        for (int g = 0; g < 4; ++g) {
          int p[16], w[16];
          for (int l = 0; l < 16; ++l) p[l] = ren[pl.CACC + a[16 * g + l]], w[l] = ren[pl.W + a[16 * g + l]];
          c += write_cost_s(p, 16) + write_cost_s(w, 16);
        }
        for (int h = 0; h < 2; ++h) {
          int p[32];
          for (int l = 0; l < 32; ++l) p[l] = ren[pl.W + a[32 * h + l]];
          c += read_cost_s(p, 32, 0);
        }
      }
    };
    pass(pl.wsx, pl.RN);
    pass(pl.wsz, pl.RM);
    return c;
  }
  long total() const {
    long c = vec_cost();
    for (const Step& s : st) c += step_cost(s);
    return c;
  }

  // ---- phase A: segment positions, operand and term order, term pairing (slots fixed)
  void anneal_step(Step& s, Rng& rng, int moves) {
    // positions of the used segments per target (term pairing moves)
    std::vector<int> used;
    for (int p = 0; p < 256; ++p)
      if (s[p].t >= 0) used.push_back(p);
    if (used.empty()) return;
    int cur = step_cost(s);
    const double T0 = envd("MPCQP_T0A", 0.3), T1 = envd("MPCQP_T1A", 0.05);
    std::vector<std::array<int, 3>> groups;  // (kind, i, j) of the affected groups
    auto add_pos = [&](int p) {
      const int q = p / 64, l = p % 64;
      for (int j = 0; j < 2; ++j)
        for (int op = 0; op < 2; ++op) groups.push_back({0, (2 * q + j) * 2 + op, l / 32});
      groups.push_back({1, q, l / 16});
    };
    auto gcost = [&]() {
      std::sort(groups.begin(), groups.end());
      groups.erase(std::unique(groups.begin(), groups.end()), groups.end());
      int c = 0;
      for (auto& g : groups) c += g[0] == 0 ? rd_group(s, g[1] / 2, g[1] % 2, g[2]) : at_group(s, g[1], g[2]);
      return c;
    };
    // pair rule: segment 1 of a lane is unused or belongs to segment 0's target
    auto lane_ok = [&](int l) {
      return !pl.paired || s[64 + l].t < 0 || (s[l].t >= 0 && s[l].t == s[64 + l].t);
    };
    Step best = s;
    int bestc = cur;
    const bool no_flip = pl.mat_first || diag_env("MPCQP_NO_FLIP") != nullptr;
    for (int it = 0; it < moves; ++it) {
      if (cur < bestc) bestc = cur, best = s;
      const double T = T0 * std::pow(T1 / T0, (double)it / moves);
      const int kind = rng.below(9);
      groups.clear();
      if (kind == 8) {  // swap the pairs (segments 0 and 1) of two lanes
        const int l1 = rng.below(64), l2 = rng.below(64);
        if (l1 == l2 || (s[l1].t < 0 && s[l2].t < 0)) continue;
        for (int q = 0; q < 2; ++q) add_pos(q * 64 + l1), add_pos(q * 64 + l2);
        const int before = gcost();
        std::swap(s[l1], s[l2]), std::swap(s[64 + l1], s[64 + l2]);
        const int d = gcost() - before;
        if (d <= 0 || rng.unit() < std::exp(-d / T)) {
          cur += d;
          for (int& u : used)
            for (int q = 0; q < 2; ++q) {
              if (u == q * 64 + l1)
                u = q * 64 + l2;
              else if (u == q * 64 + l2)
                u = q * 64 + l1;
            }
        } else {
          std::swap(s[l1], s[l2]), std::swap(s[64 + l1], s[64 + l2]);
        }
      } else if (kind < 4) {  // swap two positions (at least one used)
        const int p1 = used[rng.below((int)used.size())];
        int p2 = rng.below(256);
        if (p2 == p1) continue;
        // two waves per instance: a segment stays in its wave's half (positions 0 + 1 / 2 + 3)
        if (pl.split_steps && (p1 / 128) != (p2 / 128)) continue;
        std::swap(s[p1], s[p2]);
        const bool ok = lane_ok(p1 % 64) && lane_ok(p2 % 64);
        std::swap(s[p1], s[p2]);
        if (!ok) continue;
        add_pos(p1), add_pos(p2);
        const int before = gcost();
        std::swap(s[p1], s[p2]);
        const int d = gcost() - before;
        if (d <= 0 || rng.unit() < std::exp(-d / T)) {
          cur += d;
          for (int& u : used) {
            if (u == p1)
              u = p2;
            else if (u == p2)
              u = p1;
          }
        } else {
          std::swap(s[p1], s[p2]);
        }
      } else if (kind < 6) {  // flip the operands of one term
        // Plan::mat_first (or MPCQP_NO_FLIP, diagnostics): keep every term's matrix operand first
        // (a = matrix, b = vector), the convention the matrix-operand prefetch of the solve steps
        // relies on
        if (no_flip) continue;
        const int p = used[rng.below((int)used.size())], j = rng.below(2);
        if (s[p].a[j] < 0) continue;
        const int q = p / 64, l = p % 64;
        for (int op = 0; op < 2; ++op) groups.push_back({0, (2 * q + j) * 2 + op, l / 32});
        const int before = gcost();
        std::swap(s[p].a[j], s[p].b[j]);
        const int d = gcost() - before;
        if (d <= 0 || rng.unit() < std::exp(-d / T))
          cur += d;
        else
          std::swap(s[p].a[j], s[p].b[j]);
      } else {  // swap two terms of one target (same or another segment)
        const int p1 = used[rng.below((int)used.size())];
        const int p2 = used[rng.below((int)used.size())];
        if (s[p1].t != s[p2].t) continue;
        const int j1 = rng.below(2), j2 = rng.below(2);
        if (p1 == p2 && j1 == j2) continue;
        add_pos(p1), add_pos(p2);
        const int before = gcost();
        std::swap(s[p1].a[j1], s[p2].a[j2]);
        std::swap(s[p1].b[j1], s[p2].b[j2]);
        const int d = gcost() - before;
        if (d <= 0 || rng.unit() < std::exp(-d / T)) {
          cur += d;
        } else {
          std::swap(s[p1].a[j1], s[p2].a[j2]);
          std::swap(s[p1].b[j1], s[p2].b[j2]);
        }
      }
    }
    if (cur < bestc) bestc = cur, best = s;
    s = best;
    // a segment whose two terms both became padding adds nothing: unused (its target frees a bank)
    // -- unless it is segment 0 of a pair whose segment 1 is used (that sum needs the atomic)
    for (int p = 0; p < 256; ++p) {
      Seg& g = s[p];
      if (g.t >= 0 && g.a[0] < 0 && g.a[1] < 0 && !(pl.paired && p < 64 && s[64 + p].t >= 0)) g.t = -1;
    }
  }

  // ---- phase B: slot permutations (positions fixed)
  // groups: kind 0 read (with zero-padding count), 1 write/atomic; members are slots (names)
  struct Group {
    int kind, nz;
    std::vector<int> mem;
    int cost;
  };
  std::vector<Group> G;
  std::vector<std::vector<int>> occ;  // slot -> groups
  int gcost(const Group& g) const {
    int a[64];
    for (size_t i = 0; i < g.mem.size(); ++i) a[i] = ren[g.mem[i]];
    return g.kind == 0 ? read_cost_s(a, (int)g.mem.size(), g.nz) : write_cost_s(a, (int)g.mem.size());
  }
  void build_groups() {
    G.clear();
    occ.assign(ren.size(), {});
    for (const Step& s : st) {
      for (int c = 0; c < 8; ++c)
        for (int op = 0; op < 2; ++op)
          for (int h = 0; h < 2; ++h) {
            Group g{0, 0, {}, 0};
            for (int l = 32 * h; l < 32 * h + 32; ++l) {
              const Seg& x = s[(c / 2) * 64 + l];
              const int v = op ? x.b[c % 2] : x.a[c % 2];
              if (v < 0)
                g.nz++;
              else
                g.mem.push_back(v);
            }
            G.push_back(std::move(g));
          }
      for (int q = 0; q < 4; ++q) {
        if (q == 1 && pl.paired) continue;  // summed into segment 0's atomic
        for (int grp = 0; grp < 4; ++grp) {
          Group g{1, 0, {}, 0};
          for (int l = 16 * grp; l < 16 * grp + 16; ++l)
            if (s[q * 64 + l].t >= 0) g.mem.push_back(s[q * 64 + l].t);
          G.push_back(std::move(g));
        }
      }
    }
    auto pass = [&](const std::vector<uint16_t>& ws, int slots) {
      for (int r = 0; r < slots; ++r) {
        for (int grp = 0; grp < 4; ++grp) {
          Group g{1, 0, {}, 0}, gw{1, 0, {}, 0};
          for (int l = 16 * grp; l < 16 * grp + 16; ++l) {
            g.mem.push_back(pl.CACC + ws[64 * r + l] - pl.W);
            gw.mem.push_back(ws[64 * r + l]);
          }
          G.push_back(std::move(g));
          G.push_back(std::move(gw));
        }
        for (int h = 0; h < 2; ++h) {
          Group g{0, 0, {}, 0};
          for (int l = 32 * h; l < 32 * h + 32; ++l) g.mem.push_back(ws[64 * r + l]);
          G.push_back(std::move(g));
        }
      }
    };
    pass(pl.wsx, pl.RN);
    pass(pl.wsz, pl.RM);
    for (size_t i = 0; i < G.size(); ++i) {
      for (int x : G[i].mem) {
        auto& o = occ[x];
        if (o.empty() || o.back() != (int)i) o.push_back((int)i);
      }
      G[i].cost = gcost(G[i]);
    }
  }
  void anneal_slots(Rng& rng, int moves) {
    build_groups();
    const int nlive = pl.nLlive, nb0 = pl.NB, nM = pl.ZERO - pl.NB, NKP = pl.NKP;
    auto inL = [&](int x) { return x >= pl.LX && x < pl.LX + pl.nnzL; };
    const double T0 = envd("MPCQP_T0B", 0.5), T1 = envd("MPCQP_T1B", 0.05);
    std::vector<int> gs, names;
    std::vector<int> saved;
    long cur = 0;
    for (const Group& g : G) cur += g.cost;
    long bestc = cur;
    std::vector<int> best = ren;
    for (int it = 0; it < moves; ++it) {
      const double T = T0 * std::pow(T1 / T0, (double)it / moves);
      const int kind = rng.below(3);
      names.clear();
      int x1, x2;  // the swapped name sets are names[0..k) <-> names[k..2k)
      if (kind == 0) {  // two L-live slots
        if (nlive < 2) continue;
        x1 = pl.LX + rng.below(nlive), x2 = pl.LX + rng.below(nlive);
        if (x1 == x2) continue;
        names = {x1, x2};
      } else if (kind == 1) {  // two N | G | G' slots
        if (nM < 2) continue;
        x1 = nb0 + rng.below(nM), x2 = nb0 + rng.below(nM);
        if (x1 == x2) continue;
        names = {x1, x2};
      } else {  // two vector entries (W, C and 1/D move together)
        const int k1 = rng.below(NKP), k2 = rng.below(NKP);
        if (k1 == k2 || inL(pl.W + k1) != inL(pl.W + k2) || inL(pl.CACC + k1) != inL(pl.CACC + k2))
          continue;
        names = {pl.W + k1, pl.CACC + k1, pl.DINV + k1, pl.W + k2, pl.CACC + k2, pl.DINV + k2};
      }
      gs.clear();
      for (int x : names)
        for (int g : occ[x]) gs.push_back(g);
      std::sort(gs.begin(), gs.end());
      gs.erase(std::unique(gs.begin(), gs.end()), gs.end());
      const size_t k = names.size() / 2;
      auto swp = [&]() {
        for (size_t i = 0; i < k; ++i) std::swap(ren[names[i]], ren[names[k + i]]);
      };
      long before = 0, after = 0;
      for (int g : gs) before += G[g].cost;
      swp();
      saved.resize(gs.size());
      for (size_t i = 0; i < gs.size(); ++i) after += (saved[i] = gcost(G[gs[i]]));
      const long d = after - before;
      if (d <= 0 || rng.unit() < std::exp(-d / T)) {
        for (size_t i = 0; i < gs.size(); ++i) G[gs[i]].cost = saved[i];
        cur += d;
        if (cur < bestc) bestc = cur, best = ren;
      } else {
        swp();
      }
    }
    ren = best;
  }

  // ---- read the plan's solve tables / write them back with the renaming applied
  void load() {
    ren.resize(pl.LDS_N);
    for (int i = 0; i < pl.LDS_N; ++i) ren[i] = i;
    const int z0 = pl.ZERO, z1 = pl.ZERO + ZERO_BLOCK;
    auto isz = [&](uint32_t w) { return (int)(w / 8u) >= z0 && (int)(w / 8u) < z1; };
    // sinks: targets of all-zero segments
    for (int w = 0; w < 2; ++w) {
      const auto& t = w ? pl.bwd : pl.fwd;
      const int ns = w ? pl.nbwd : pl.nfwd;
      for (int s = 0; s < ns; ++s) {
        const uint32_t* r = t.data() + (size_t)s * SOLVE_STEP_WORDS;
        Step S;
        for (int q = 0; q < 4; ++q)
          for (int l = 0; l < 64; ++l) {
            const uint32_t* x = r + q * 256 + l * 4;
            Seg g;
            for (int j = 0; j < 2; ++j) {
              const bool pad = isz(x[2 * j]) || isz(x[2 * j + 1]);
              g.a[j] = pad ? -1 : (int)(x[2 * j] / 8u);
              g.b[j] = pad ? -1 : (int)(x[2 * j + 1] / 8u);
            }
            if (g.a[0] >= 0 || g.a[1] >= 0) g.t = (int)(r[SOLVE_TERM_WORDS + l * 4 + q] / 8u);
            S[q * 64 + l] = g;
          }
        st.push_back(S);
      }
    }
  }
  void store() {
    const uint32_t zb = (uint32_t)pl.ZERO;
    // zero slot of the least used bank per read group; sinks in free banks per atomic group
    // sinks: the 1/D region's padding slots (construction slots nk..NKP-1, renamed), which hold 0
    // and are only ever multiplied by the zero W padding; an idle segment adds -0.0 (exact no-op).
    // Should the padding not cover every bank, the live 1/D slots of the missing banks join the
    // pool (still exact: adding -0.0 never changes a value)
    std::vector<int> sinkpool[WBANKS];
    for (int k = pl.nk; k < pl.NKP; ++k) {
      const int slot = ren[pl.DINV + k];
      sinkpool[slot & (WBANKS - 1)].push_back(slot);
    }
    for (int k = 0; k < pl.NKP; ++k) {
      const int slot = ren[pl.DINV + k];
      if (sinkpool[slot & (WBANKS - 1)].empty()) sinkpool[slot & (WBANKS - 1)].push_back(slot);
    }
    size_t si = 0;
    for (int w = 0; w < 2; ++w) {
      auto& t = w ? pl.bwd : pl.fwd;
      const int ns = w ? pl.nbwd : pl.nfwd;
      for (int s = 0; s < ns; ++s, ++si) {
        const Step& S = st[si];
        uint32_t* r = t.data() + (size_t)s * SOLVE_STEP_WORDS;
        for (int c = 0; c < 8; ++c)
          for (int op = 0; op < 2; ++op)
            for (int h = 0; h < 2; ++h) {
              int nb[RBANKS] = {};
              std::vector<int> seen;
              const int q = c / 2, j = c % 2;
              for (int l = 32 * h; l < 32 * h + 32; ++l) {
                const Seg& g = S[q * 64 + l];
                const int x = op ? g.b[j] : g.a[j];
                if (x >= 0 && std::find(seen.begin(), seen.end(), ren[x]) == seen.end())
                  seen.push_back(ren[x]), nb[ren[x] & (RBANKS - 1)]++;
              }
              int best = 0;
              for (int b = 1; b < RBANKS; ++b)
                if (nb[b] < nb[best]) best = b;
              // zero slot on bank `best`
              const uint32_t zslot = zb + (uint32_t)((best - (int)(zb & (RBANKS - 1)) + RBANKS) & (RBANKS - 1));
              for (int l = 32 * h; l < 32 * h + 32; ++l) {
                const Seg& g = S[q * 64 + l];
                const int x = op ? g.b[j] : g.a[j];
                r[q * 256 + l * 4 + 2 * j + op] = (x >= 0 ? (uint32_t)ren[x] : zslot) * 8u;
              }
            }
        for (int q = 0; q < 4; ++q)
          for (int grp = 0; grp < 4; ++grp) {
            if (q == 1 && pl.paired) continue;  // segment 1 of a pair: no atomic (its word repeats t0 below)
            int c[WBANKS] = {};
            for (int l = 16 * grp; l < 16 * grp + 16; ++l)
              if (S[q * 64 + l].t >= 0) c[ren[S[q * 64 + l].t] & (WBANKS - 1)]++;
            int nextb = 0;
            for (int l = 16 * grp; l < 16 * grp + 16; ++l) {
              const int tt = S[q * 64 + l].t;
              uint32_t slot;
              if (tt >= 0) {
                slot = (uint32_t)ren[tt];
              } else {
                while (c[nextb]) ++nextb;  // a free bank exists: 16 lanes, 16 banks
                c[nextb] = 1;
                slot = (uint32_t)sinkpool[nextb][l % sinkpool[nextb].size()];
              }
              r[SOLVE_TERM_WORDS + l * 4 + q] = slot * 8u;
            }
          }
        if (pl.paired)
          for (int l = 0; l < 64; ++l) r[SOLVE_TERM_WORDS + l * 4 + 1] = r[SOLVE_TERM_WORDS + l * 4 + 0];
      }
    }
    // every other table: relabel slots
    auto mp = [&](uint32_t byteaddr) { return (uint32_t)ren[byteaddr / 8u] * 8u; };
    for (int w = 0; w < 2; ++w) {
      auto& t = w ? pl.tail : pl.fac;
      const int ns = w ? pl.ntail : pl.nfac;
      for (int s = 0; s < ns; ++s) {
        uint32_t* r = t.data() + (size_t)s * FAC_STEP_WORDS;
        for (int l = 0; l < 64; ++l)
          if (r[l] & META_HEAD) r[l] = (r[l] & ~META_TGT_MASK) | mp(r[l] & META_TGT_MASK);
        for (int k = 64; k < FAC_STEP_WORDS; ++k) r[k] = mp(r[k]);
      }
    }
    auto mp16 = [&](std::vector<uint16_t>& v) {
      for (auto& x : v) x = (uint16_t)ren[x];
    };
    mp16(pl.slotP), mp16(pl.slotA), mp16(pl.slotRho), mp16(pl.slotSig), mp16(pl.wsx), mp16(pl.wsz);
    std::vector<uint16_t> lc(pl.nnzL);
    for (int k = 0; k < pl.nnzL; ++k) lc[ren[pl.LX + k] - pl.LX] = (uint16_t)ren[pl.Lcol[k]];
    pl.Lcol.swap(lc);
  }
};

}  // namespace

LdsModel model_lds(const Plan& pl) {
  LdsModel m;
  for (int w = 0; w < 2; ++w) {
    const auto& t = w ? pl.bwd : pl.fwd;
    const int ns = w ? pl.nbwd : pl.nfwd;
    for (int s = 0; s < ns; ++s) {
      const uint32_t* r = t.data() + (size_t)s * SOLVE_STEP_WORDS;
      for (int c = 0; c < 8; ++c)
        for (int op = 0; op < 2; ++op)
          for (int h = 0; h < 2; ++h) {
            int a[32];
            for (int l = 0; l < 32; ++l) a[l] = (int)(r[(c / 2) * 256 + (32 * h + l) * 4 + (c % 2) * 2 + op] / 8u);
            m.read += read_cost(a, 32, 0);
          }
      for (int q = 0; q < 4; ++q)
        for (int g = 0; g < 4; ++g) {
          if (q == 1 && pl.paired) continue;  // segments 0 + 1 share one atomic
          int a[16];
          for (int l = 0; l < 16; ++l) a[l] = (int)(r[SOLVE_TERM_WORDS + (16 * g + l) * 4 + q] / 8u);
          m.atomic += write_cost(a, 16);
        }
      m.floor += 32 + (pl.paired ? 12 : 16);
    }
  }
  auto pass = [&](const std::vector<uint16_t>& ws, int slots) {
    for (int r = 0; r < slots; ++r) {
      for (int g = 0; g < 4; ++g) {
        int a[16], w[16];
        for (int l = 0; l < 16; ++l) a[l] = pl.CACC - pl.W + ws[64 * r + 16 * g + l], w[l] = ws[64 * r + 16 * g + l];
        m.vec += write_cost(a, 16) + write_cost(w, 16);
      }
      for (int h = 0; h < 2; ++h) {
        int a[32];
        for (int l = 0; l < 32; ++l) a[l] = ws[64 * r + 32 * h + l];
        m.vec += read_cost(a, 32, 0);
      }
      m.floor += 10;
    }
  };
  pass(pl.wsx, pl.RN);
  pass(pl.wsz, pl.RM);
  return m;
}

void optimize_lds(Plan& pl) {
  if ((int)pl.wsx.size() != 64 * pl.RN || (int)pl.wsz.size() != 64 * pl.RM) return;
  Opt o(pl);
  o.load();
  Rng rng(0x5eed);
  const double scale = std::max(0.25, std::min(4.0, atof(diag_env("MPCQP_ANNEAL_SCALE") ? diag_env("MPCQP_ANNEAL_SCALE") : "1")));
  const long c0 = o.total();
  const bool dbg = diag_env("MPCQP_DUMP_CONFLICTS") != nullptr;
  for (int round = 0; round < 3; ++round) {
    for (Step& s : o.st) {
      const int b = dbg ? o.step_cost(s) : 0;
      o.anneal_step(s, rng, (int)(20000 * scale));
      if (dbg) fprintf(stderr, "  step: %d -> %d\n", b, o.step_cost(s));
    }
    const long b = dbg ? o.total() : 0;
    o.anneal_slots(rng, (int)(60000 * scale * o.st.size() / 13.0));
    if (dbg) fprintf(stderr, " slots: %ld -> %ld\n", b, o.total());
  }
  for (Step& s : o.st) o.anneal_step(s, rng, (int)(20000 * scale));
  const long c1 = o.total();
  if (dbg) {  // segments per target per step, atomic excess per step
    for (const Step& S : o.st) {
      std::vector<int> cnt(pl.LDS_N, 0);
      int mx = 0, nt = 0, nu = 0;
      for (const Seg& g : S)
        if (g.t >= 0) nu++, mx = std::max(mx, ++cnt[g.t]);
      for (int c : cnt) nt += c > 0;
      int ex = 0;
      for (int q = 0; q < 4; ++q)
        for (int gg = 0; gg < 4; ++gg) ex += o.at_group(S, q, gg) / SM - 1;
      fprintf(stderr, "  step: %d used segs, %d targets, max segs/target %d, atomic excess %d\n", nu, nt, mx, ex);
    }
  }
  if (diag_env("MPCQP_DUMP_CONFLICTS")) fprintf(stderr, "optimize_lds: modelled cycles %ld -> %ld\n", c0, c1);
  o.store();
}

}  // namespace mpcqp
