// plan_stats.cpp -- host diagnostic: the engine's compiled plan for a QP structure (solve-step
// occupancy, operand classes, LDS regions).  Build: g++ -O2 -std=c++17 tools/plan_stats.cpp
// mpc_arpo_project_amd/csrc/symbolic.cpp mpc_arpo_project_amd/csrc/lds_layout.cpp -o /tmp/plan_stats
// Input: "n m nnzP nnzA" then the Pp, Pi, Ap, Ai lines (CSC, P upper triangle).
#include <cstdio>
#include <cstdlib>
#include <map>
#include <set>
#include <algorithm>
#include <vector>

#include "../mpc_arpo_project_amd/csrc/symbolic.hpp"

using namespace mpcqp;

static std::vector<int32_t> rd(FILE* f, int cnt) {
  std::vector<int32_t> v(cnt);
  for (int i = 0; i < cnt; i++)
    if (fscanf(f, "%d", &v[i]) != 1) exit(2);
  return v;
}

int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "r");
  int n, m, nP, nA;
  if (fscanf(f, "%d %d %d %d", &n, &m, &nP, &nA) != 4) return 2;
  auto Pp = rd(f, n + 1), Pi = rd(f, nP), Ap = rd(f, n + 1), Ai = rd(f, nA);
  Plan pl;
  const int capM = argc > 2 ? atoi(argv[2]) : 0, capW = argc > 3 ? atoi(argv[3]) : 0;
  if (!build_plan_tuned(n, m, Pp.data(), Pi.data(), Ap.data(), Ai.data(), pl, capM, capW)) {
    printf("error %s\n", pl.error.c_str());
    return 1;
  }
  const int nk = n + m;
  printf("n %d m %d nk %d nnzL %d nLlive %d nN %d nG %d nGP %d blocks %zu paired %d\n", n, m, nk,
         pl.nnzL, pl.nLlive, pl.nN, pl.nG, pl.nGP, pl.block_start.size() - 1, (int)pl.paired);
  printf("blocks:");
  for (size_t k = 0; k + 1 < pl.block_start.size(); k++)
    printf(" %d", pl.block_start[k + 1] - pl.block_start[k]);
  printf("\nLDS image %d B; fac %d tail %d fwd %d bwd %d steps\n", pl.LDS_N * 8, pl.nfac, pl.ntail,
         pl.nfwd, pl.nbwd);
  printf("fwd steps per level:");
  for (int x : pl.fwd_level_steps) printf(" %d", x);
  printf("\nbwd steps per level:");
  for (int x : pl.bwd_level_steps) printf(" %d", x);
  printf("\n");
  auto is_vec = [&](uint32_t byte) {
    const int s = (int)(byte / 8);
    return (s >= pl.W && s < pl.W + pl.NKP) || (s >= pl.CACC && s < pl.CACC + pl.NKP);
  };
  const int zero_lo = pl.ZERO, zero_hi = pl.ZERO + ZERO_BLOCK;
  for (int dir = 0; dir < 2; dir++) {
    const auto& t = dir ? pl.bwd : pl.fwd;
    const int ns = dir ? pl.nbwd : pl.nfwd;
    std::set<uint32_t> mats;
    long used_terms = 0, used_segs = 0, pair_adj = 0;
    for (int s = 0; s < ns; s++) {
      const uint32_t* st = t.data() + (size_t)s * SOLVE_STEP_WORDS;
      int seg_used = 0, terms = 0;
      for (int l = 0; l < 64; l++)
        for (int q = 0; q < SOLVE_MAXC / 2; q++) {
          const uint32_t* w = st + q * 256 + l * 4;  // (a0, b0, a1, b1) of segment q
          int segterms = 0;
          uint32_t mt[2] = {0, 0};
          for (int h = 0; h < 2; h++) {
            const uint32_t a = w[2 * h], b = w[2 * h + 1];
            const int sa = a / 8, sb = b / 8;
            const bool za = sa >= zero_lo && sa < zero_hi, zb = sb >= zero_lo && sb < zero_hi;
            if (za || zb) continue;
            segterms++;
            const uint32_t mat = is_vec(a) ? b : a;
            mats.insert(mat);
            mt[h] = mat;
          }
          terms += segterms;
          if (segterms) seg_used++;
          if (segterms == 2 && (mt[0] + 8 == mt[1] || mt[1] + 8 == mt[0])) pair_adj++;
        }
      printf("  %s step %2d: segments %3d / 256, terms %3d / 512\n", dir ? "bwd" : "fwd", s, seg_used,
             terms);
      used_terms += terms, used_segs += seg_used;
    }
    printf("%s: %ld segments, %ld terms, %zu distinct matrix slots, adjacent matrix pairs %ld\n",
           dir ? "bwd" : "fwd", used_segs, used_terms, mats.size(), pair_adj);
  }
  // per-target term counts of the last backward level (steps from the last level's start)
  {
    int first = pl.nbwd - pl.bwd_level_steps.back();
    std::map<uint32_t, std::pair<int, int>> tg;  // target -> (terms, MONE terms)
    const uint32_t mone = (uint32_t)pl.MONE * 8;
    for (int s = first; s < pl.nbwd; s++) {
      const uint32_t* st = pl.bwd.data() + (size_t)s * SOLVE_STEP_WORDS;
      for (int l = 0; l < 64; l++) {
        const uint32_t* tq = st + SOLVE_TERM_WORDS + l * 4;
        for (int q = 0; q < 4; q++) {
          const uint32_t t = (q == 1 && pl.paired) ? tq[0] : tq[q];
          const uint32_t* w = st + q * 256 + l * 4;
          for (int h = 0; h < 2; h++) {
            const uint32_t a = w[2 * h], b = w[2 * h + 1];
            const int sa = a / 8, sb = b / 8;
            if ((sa >= zero_lo && sa < zero_hi) || (sb >= zero_lo && sb < zero_hi)) continue;
            tg[t].first++;
            if (a == mone || b == mone) tg[t].second++;
          }
        }
      }
    }
    // C targets hit by earlier backward steps (far-block accumulations)
    std::set<uint32_t> acc;
    for (int s = 0; s < first; s++) {
      const uint32_t* st = pl.bwd.data() + (size_t)s * SOLVE_STEP_WORDS;
      for (int l = 0; l < 64; l++)
        for (int q = 0; q < 4; q++) acc.insert(st[SOLVE_TERM_WORDS + l * 4 + q]);
    }
    int fin = 0, fin_only = 0, seg_now = 0, seg_new = 0;
    for (auto& kv : tg) {
      const bool final_c = !acc.count(kv.first + (uint32_t)pl.NKP * 8);
      const int t = kv.second.first;
      seg_now += (t + 1) / 2;
      if (final_c) {
        fin++;
        if (t == kv.second.second) fin_only++;
        seg_new += t / 2;  // the MONE term folded into the target's initial value
      } else {
        seg_new += (t + 1) / 2;
      }
    }
    printf("last bwd level: %d targets with a final C at the diagonal pass (%d of them copies); "
           "segments (unpaired count) %d -> %d\n", fin, fin_only, seg_now, seg_new);
    int only_mone = 0, hist[8] = {};
    for (auto& kv : tg) {
      if (kv.second.first == kv.second.second) only_mone++;
      hist[std::min(kv.second.first, 7)]++;
    }
    printf("last bwd level: %zu targets, %d with only the MONE term; terms/target histogram:", tg.size(),
           only_mone);
    for (int i = 0; i < 8; i++) printf(" %d:%d", i, hist[i]);
    printf("\n");
  }
  return 0;
}
