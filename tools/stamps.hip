// Diagnostics: per-wave phase timeline of one be_step launch (needs the -DBE_DIAG_STAMPS library in tools/diag).
// build: hipcc --offload-arch=gfx950 -O3 -I include tools/stamps.hip -L tools/diag -lballenv -Wl,-rpath,'$ORIGIN/diag' -o tools/stamps
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>
#include "ballenv.h"
extern "C" int be_diag_stamps(unsigned long long* rt, unsigned long long* cy);
extern "C" int be_diag_clear(void);
extern "C" int be_diag_hwid(unsigned int* hw);
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
constexpr int DW = 1 << 16, DP = 16;
static double pct(std::vector<double> v, double p) { if (v.empty()) return 0; std::sort(v.begin(), v.end()); return v[(size_t)(p * (v.size() - 1))]; }
int main(int argc, char** argv) {
  int N = argc > 1 ? atoi(argv[1]) : 65536;
  be_config cfg; be_config_default(&cfg, N, 10);
  be_ctx* ctx = nullptr;
  if (be_create(&cfg, 0, &ctx)) { printf("create: %s\n", be_last_error(nullptr)); return 1; }
  be_state st; be_out out; memset(&st, 0, sizeof st); memset(&out, 0, sizeof out);
  CK(hipMalloc(&st.agent, 4 * N)); CK(hipMalloc(&st.goal, 4 * N)); CK(hipMalloc(&st.prev_dist, 8 * N));
  CK(hipMalloc(&st.total_dist, 8 * N)); CK(hipMalloc(&st.ep_return, 8 * N)); CK(hipMalloc(&st.ep_len, 4 * N));
  CK(hipMalloc(&st.episode, 4 * N)); CK(hipMalloc(&st.static_obs, 4 * 13 * N)); CK(hipMalloc(&st.dyn_obs, 4 * 5 * N));
  CK(hipMalloc(&st.dyn_goal, 5 * N)); CK(hipMalloc(&out.obs, 104 * N)); CK(hipMalloc(&out.reward, 8 * N)); CK(hipMalloc(&out.done, N));
  CK(hipMemset(st.episode, 0, 4 * N)); CK(hipMemset(st.ep_len, 0, 4 * N));
  uint8_t* acts; CK(hipMalloc(&acts, (size_t)N * 64));
  be_sample_actions(ctx, acts, 64, 7, nullptr);
  be_reset(ctx, &st, nullptr, nullptr, 0, &out, nullptr);
  for (int k = 0; k < 300; ++k) be_step(ctx, &st, acts + (size_t)(k % 64) * N, nullptr, nullptr, &out, nullptr);
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> rt(DW * DP), cy(DW * DP);
  for (int rep = 0; rep < 3; ++rep) {
    // rep 0: one cold launch after a sync; reps 1, 2: the last of 20 back-to-back launches
    be_diag_clear();
    for (int k = 0; k < (rep == 0 ? 1 : 20); ++k)
      be_step(ctx, &st, acts + (size_t)((rep * 20 + k) % 64) * N, nullptr, nullptr, &out, nullptr);
    CK(hipDeviceSynchronize());
    be_diag_stamps(rt.data(), cy.data());
    int waves = 0; unsigned long long t0 = ~0ull, t1 = 0;
    for (int w = 0; w < DW; ++w) if (rt[w * DP + 0]) { waves++; t0 = std::min(t0, rt[w * DP + 0]); t1 = std::max(t1, rt[w * DP + 6]); }
    std::vector<double> start, endt; std::vector<std::vector<double>> ph(6);
    for (int w = 0; w < DW; ++w) {
      if (!rt[w * DP + 0]) continue;
      start.push_back((rt[w * DP + 0] - t0) * 0.01); endt.push_back((rt[w * DP + 6] - t0) * 0.01);
      for (int p = 0; p < 6; ++p) ph[p].push_back((double)(cy[w * DP + p + 1] - cy[w * DP + p]));
    }
    printf("rep %d: N=%d waves=%d span(first start..last end)=%.2f us\n", rep, N, waves, (t1 - t0) * 0.01);
    if (rep == 2) {   // where the waves ran: per XCD start spread, blocks per CU
      std::vector<unsigned> hw(DW);
      be_diag_hwid(hw.data());
      std::vector<std::vector<double>> xs(16);
      std::vector<int> per_cu(16 * 4 * 2 * 16, 0);
      for (int w = 0; w < DW; ++w) {
        if (!rt[w * DP + 0]) continue;
        const unsigned h = hw[w], xcc = h >> 28, cu = (h >> 8) & 15, sh = (h >> 12) & 1, se = (h >> 13) & 3;
        xs[xcc & 15].push_back((rt[w * DP + 0] - t0) * 0.01);
        if ((w & 3) == 0) per_cu[(((xcc & 15) * 4 + se) * 2 + sh) * 16 + cu]++;   // one count per block (4 waves)
      }
      for (int x = 0; x < 16; ++x)
        if (!xs[x].empty())
          printf("  xcc %d: waves %zu start p0 %.2f p50 %.2f max %.2f us\n", x, xs[x].size(), pct(xs[x], 0), pct(xs[x], .5), pct(xs[x], 1));
      std::vector<int> hist(8, 0);
      int used = 0;
      for (int c : per_cu) { if (c) { used++; hist[std::min(c, 7)]++; } }
      printf("  CUs used %d; blocks per used CU histogram:", used);
      for (int k = 1; k < 8; ++k) printf(" %d:%d", k, hist[k]);
      printf("\n");
    }
    printf("  wave start us: p0 %.2f p50 %.2f p90 %.2f max %.2f | wave end us: p10 %.2f p50 %.2f p90 %.2f max %.2f\n",
           pct(start, 0), pct(start, .5), pct(start, .9), pct(start, 1), pct(endt, .1), pct(endt, .5), pct(endt, .9), pct(endt, 1));
    const char* names[6] = {"entry->barrier1 (loads)", "barrier1->physics", "physics->reset list", "list->stage written", "stage->after coop reset", "coop reset->end(copy)"};
    for (int p = 0; p < 6; ++p)
      printf("  %-26s cycles p50 %8.0f p90 %8.0f p99 %8.0f max %8.0f\n", names[p], pct(ph[p], .5), pct(ph[p], .9), pct(ph[p], .99), pct(ph[p], 1));
    std::vector<std::vector<double>> sub(5);
    for (int w = 0; w < DW; ++w) {
      const unsigned long long* c = &cy[w * DP];
      // step2_kernel stamps 1 -> 7 (counter, Philox) -> 11 (dynamic moves) -> 8 (action, move,
      // distance) -> 10 (obstacle tests) -> 2 (reward, stores)
      if (!rt[w * DP + 0] || !(c[7] > c[1] && c[11] >= c[7] && c[8] >= c[11] && c[10] >= c[8] && c[2] >= c[10])) continue;
      sub[0].push_back((double)(c[7] - c[1])); sub[1].push_back((double)(c[11] - c[7]));
      sub[2].push_back((double)(c[8] - c[11])); sub[3].push_back((double)(c[10] - c[8]));
      sub[4].push_back((double)(c[2] - c[10]));
    }
    const char* sn[5] = {"  physics: counter+philox", "  physics: dynamic moves", "  physics: action+distance",
                         "  physics: obstacle tests", "  physics: reward+stores"};
    for (int p = 0; p < 5; ++p)
      if (!sub[p].empty())
        printf("  %-26s cycles p50 %8.0f p90 %8.0f p99 %8.0f max %8.0f\n", sn[p], pct(sub[p], .5), pct(sub[p], .9), pct(sub[p], .99), pct(sub[p], 1));
    // fixed-shape kernels: 8 -> 7 Philox, 7 -> 11 dynamic moves + their tests, 11 -> 9 static tests
    std::vector<std::vector<double>> fx(3);
    for (int w = 0; w < DW; ++w) {
      if (!rt[w * DP + 0] || !cy[w * DP + 7] || !cy[w * DP + 11] || cy[w * DP + 8] > cy[w * DP + 7]) continue;   // be_kernel order
      fx[0].push_back((double)(cy[w * DP + 7] - cy[w * DP + 8]));
      fx[1].push_back((double)(cy[w * DP + 11] - cy[w * DP + 7]));
      fx[2].push_back((double)((cy[w * DP + 9] ? cy[w * DP + 9] : cy[w * DP + 10]) - cy[w * DP + 11]));
    }
    // waves that ran resets in THIS launch: coop (generic): 4 -> 12 phase A, 12 -> 13 B, 13 -> 14 C;
    // wave resets (fixed-shape): 2 -> 12 draws, 12 -> 13 obstacles + raster, 13 -> 14 owner stores
    std::vector<std::vector<double>> cr(3);
    for (int w = 0; w < DW; ++w) {
      const unsigned long long* r = &rt[w * DP];
      if (!r[0] || r[12] < r[0] || r[12] > r[6] || r[14] < r[13]) continue;
      const unsigned long long* c = &cy[w * DP];
      cr[0].push_back((double)(c[12] - (c[12] > c[4] ? c[4] : c[2]))); cr[1].push_back((double)(c[13] - c[12])); cr[2].push_back((double)(c[14] - c[13]));
    }
    const char* cn[3] = {"    coop: barrier+phase A", "    coop: phase B", "    coop: phase C"};
    if (!cr[0].empty()) printf("  coop-reset waves: %zu\n", cr[0].size());
    for (int p = 0; p < 3; ++p)
      if (!cr[p].empty())
        printf("  %-26s cycles p50 %8.0f p90 %8.0f p99 %8.0f max %8.0f\n", cn[p], pct(cr[p], .5), pct(cr[p], .9), pct(cr[p], .99), pct(cr[p], 1));
    {   // BALLENV_DEBUG_SKIP=1024: barrier 1 -> every load landed
      std::vector<double> la;
      for (int w = 0; w < DW; ++w) {
        const unsigned long long* r = &rt[w * DP];
        if (r[0] && r[15] >= r[0] && r[15] <= r[6]) la.push_back((double)(cy[w * DP + 15] - cy[w * DP + 1]));
      }
      if (!la.empty())
        printf("  %-26s cycles p50 %8.0f p90 %8.0f p99 %8.0f max %8.0f\n", "  barrier1 -> loads landed", pct(la, .5), pct(la, .9), pct(la, .99), pct(la, 1));
    }
    const char* fn[3] = {"    fixed: counter+philox", "    fixed: dyn moves", "    fixed: static tests"};
    for (int p = 0; p < 3; ++p)
      if (!fx[p].empty())
        printf("  %-26s cycles p50 %8.0f p90 %8.0f p99 %8.0f max %8.0f\n", fn[p], pct(fx[p], .5), pct(fx[p], .9), pct(fx[p], .99), pct(fx[p], 1));
    if (rep == 2) {   // the tail: which waves end last, and where their time went
      std::vector<unsigned> hw(DW);
      be_diag_hwid(hw.data());
      std::vector<int> idx;
      for (int w = 0; w < DW; ++w) if (rt[w * DP + 0]) idx.push_back(w);
      std::sort(idx.begin(), idx.end(), [&](int a, int b) { return rt[a * DP + 6] > rt[b * DP + 6]; });
      std::vector<double> end_r, end_n, end_p, hit_wait;
      std::vector<std::vector<double>> end_x(16);
      // POOL_STAMP=1 (step2_kernel<..., true>): stamp 9 = a pool entry landed in this launch (a hit wave)
      const bool pool_stamp = getenv("POOL_STAMP") && atoi(getenv("POOL_STAMP"));
      for (int w : idx) {
        const unsigned long long* r = &rt[w * DP];
        const bool rs = r[12] >= r[0] && r[12] <= r[6] && r[12];
        const bool ps = pool_stamp && !rs && r[9] >= r[0] && r[9] <= r[6] && r[9];
        (rs ? end_r : ps ? end_p : end_n).push_back((r[6] - t0) * 0.01);
        if (ps) hit_wait.push_back((double)(cy[w * DP + 9] - cy[w * DP + 10]));
        end_x[(hw[w] >> 28) & 15].push_back((r[6] - t0) * 0.01);
      }
      printf("  tail: end us of reset waves (%zu) p50 %.2f max %.2f | other waves (%zu) p50 %.2f p90 %.2f p99 %.2f max %.2f\n",
             end_r.size(), end_r.empty() ? 0 : pct(end_r, .5), end_r.empty() ? 0 : pct(end_r, 1), end_n.size(), pct(end_n, .5),
             pct(end_n, .9), pct(end_n, .99), pct(end_n, 1));
      if (pool_stamp)
        printf("  tail: end us of pool-hit waves (%zu) p50 %.2f max %.2f; obstacle tests -> entry landed: cycles p50 %.0f max %.0f\n",
               end_p.size(), end_p.empty() ? 0 : pct(end_p, .5), end_p.empty() ? 0 : pct(end_p, 1),
               hit_wait.empty() ? 0 : pct(hit_wait, .5), hit_wait.empty() ? 0 : pct(hit_wait, 1));
      for (int x = 0; x < 16; ++x)
        if (!end_x[x].empty()) printf("  tail: xcc %d end p50 %.2f p90 %.2f max %.2f us\n", x, pct(end_x[x], .5), pct(end_x[x], .9), pct(end_x[x], 1));
      {   // -DBE_RESET_STAMPS builds: reset waves' phase A split (2 -> 7 -> 8 -> 9 -> 10 -> 12)
        std::vector<std::vector<double>> ra(5);
        for (int w : idx) {
          const unsigned long long* r = &rt[w * DP];
          const unsigned long long* c = &cy[w * DP];
          if (!(r[12] >= r[0] && r[12] <= r[6] && r[12]) || !(c[7] > c[2] && c[8] >= c[7] && c[9] >= c[8] && c[10] >= c[9] && c[12] >= c[10])) continue;
          ra[0].push_back((double)(c[7] - c[2])); ra[1].push_back((double)(c[8] - c[7])); ra[2].push_back((double)(c[9] - c[8]));
          ra[3].push_back((double)(c[10] - c[9])); ra[4].push_back((double)(c[12] - c[10]));
        }
        const char* rn[5] = {"stores->pass setup", "philox", "goal/agent block", "broadcast", "->stamp12"};
        if (!ra[0].empty())
          for (int q = 0; q < 5; ++q)
            printf("  reset A: %-20s cycles p50 %6.0f max %6.0f (%zu waves)\n", rn[q], pct(ra[q], .5), pct(ra[q], 1), ra[q].size());
      }
      printf("  tail: the 24 last waves (start, end us; reset; xcc/se/cu; cycles per phase 0-1 1-2 2-3 3-4 4-5 5-6)\n");
      for (int n = 0; n < 24 && n < (int)idx.size(); ++n) {
        const int w = idx[n];
        const unsigned long long* r = &rt[w * DP];
        const unsigned long long* c = &cy[w * DP];
        const unsigned h = hw[w];
        const bool rsw = r[12] >= r[0] && r[12] <= r[6] && r[12];
        const bool psw = pool_stamp && !rsw && r[9] >= r[0] && r[9] <= r[6] && r[9];
        printf("    w%5d %.2f %.2f %s x%u/se%u/cu%2u |", w, (r[0] - t0) * 0.01, (r[6] - t0) * 0.01,
               rsw ? "R" : psw ? "P" : "-", (h >> 28) & 15, (h >> 13) & 3, (h >> 8) & 15);
        for (int p = 0; p < 6; ++p) printf(" %6llu", c[p + 1] - c[p]);
        printf("\n");
      }
    }
  }
  return 0;
}
