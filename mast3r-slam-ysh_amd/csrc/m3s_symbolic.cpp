// m3s_symbolic.cpp — host symbolic analysis for the block-sparse LLT
// (see m3s_symbolic.h). Deterministic: every tie is broken by index.
#include "m3s_symbolic.h"

#include <algorithm>
#include <climits>
#include <cstdint>
#include <queue>
#include <thread>

namespace m3s {

int host_remap(const int64_t *ii, const int64_t *jj, int64_t E, std::vector<int32_t> &ri,
               std::vector<int32_t> &rj) {
  std::vector<int64_t> u(ii, ii + E);
  u.insert(u.end(), jj, jj + E);
  std::sort(u.begin(), u.end());
  u.erase(std::unique(u.begin(), u.end()), u.end());
  ri.resize(E);
  rj.resize(E);
  for (int64_t e = 0; e < E; e++) {
    ri[e] = (int32_t)(std::lower_bound(u.begin(), u.end(), ii[e]) - u.begin());
    rj[e] = (int32_t)(std::lower_bound(u.begin(), u.end(), jj[e]) - u.begin());
  }
  return (int)u.size();
}

namespace {

// Fixed-width bit rows: the variable graphs here have at most a few hundred
// vertices, so elimination updates are word-wide ORs and degrees popcounts.
struct BitRows {
  int n = 0, words = 0;
  std::vector<uint64_t> w;
  BitRows(int n_ = 0) : n(n_), words((n_ + 63) / 64), w((size_t)n_ * ((n_ + 63) / 64), 0) {}
  uint64_t *row(int r) { return w.data() + (size_t)r * words; }
  const uint64_t *row(int r) const { return w.data() + (size_t)r * words; }
  void set(int r, int c) { row(r)[c >> 6] |= uint64_t(1) << (c & 63); }
  void reset(int r, int c) { row(r)[c >> 6] &= ~(uint64_t(1) << (c & 63)); }
  bool test(int r, int c) const { return (row(r)[c >> 6] >> (c & 63)) & 1; }
  int count(int r) const {
    int k = 0;
    for (int q = 0; q < words; q++) k += __builtin_popcountll(row(r)[q]);
    return k;
  }
  template <typename F>
  void for_each(int r, F f) const {  // ascending column order
    const uint64_t *x = row(r);
    for (int q = 0; q < words; q++)
      for (uint64_t v = x[q]; v; v &= v - 1) f(q * 64 + __builtin_ctzll(v));
  }
};

// Minimum-degree elimination order on the variable graph (ties: lowest
// index). With `multiple` set, each round eliminates an independent set of
// minimum-degree (+ slack) variables together (multiple minimum degree): the
// same kind of fill, but a shallower elimination tree, i.e. fewer dependent
// steps in the dataflow factorisation.
std::vector<int32_t> min_degree_order(int m, const BitRows &adj0, bool multiple, int slack) {
  BitRows adj = adj0;
  std::vector<char> alive(m, 1);
  std::vector<int> deg(m);
  for (int v = 0; v < m; v++) deg[v] = adj.count(v);
  std::vector<int32_t> order;
  order.reserve(m);
  std::vector<int> nb;
  auto eliminate = [&](int v) {
    order.push_back(v);
    alive[v] = 0;
    nb.clear();
    adj.for_each(v, [&](int u) { nb.push_back(u); });
    const uint64_t *rv = adj.row(v);
    for (int u : nb) {
      uint64_t *ru = adj.row(u);
      for (int q = 0; q < adj.words; q++) ru[q] |= rv[q];
      adj.reset(u, u);
      adj.reset(u, v);
      deg[u] = adj.count(u);
    }
    std::fill(adj.row(v), adj.row(v) + adj.words, 0);
  };
  while ((int)order.size() < m) {
    int dmin = INT_MAX;
    for (int v = 0; v < m; v++)
      if (alive[v] && deg[v] < dmin) dmin = deg[v];
    if (!multiple) {
      for (int v = 0; v < m; v++)
        if (alive[v] && deg[v] == dmin) {
          eliminate(v);
          break;
        }
      continue;
    }
    std::vector<char> marked(m, 0);
    std::vector<int> sel;
    for (int d = dmin; d <= dmin + slack; d++)
      for (int v = 0; v < m; v++)
        if (alive[v] && !marked[v] && deg[v] == d) {
          sel.push_back(v);
          marked[v] = 1;
          adj.for_each(v, [&](int u) { marked[u] = 1; });
        }
    for (int v : sel) eliminate(v);
  }
  return order;
}

// Symbolic factorisation in elimination order: S row k = rows i > k with
// L_ik != 0 (new numbering), parent = first of them.
BitRows symbolic_fill(int m, const BitRows &adj, const std::vector<int32_t> &order,
                      std::vector<int> &parent) {
  std::vector<int32_t> pos(m);
  for (int k = 0; k < m; k++) pos[order[k]] = k;
  BitRows S(m);
  for (int v = 0; v < m; v++)
    adj.for_each(v, [&](int u) {
      if (pos[u] > pos[v]) S.set(pos[v], pos[u]);
    });
  parent.assign(m, -1);
  for (int k = 0; k < m; k++) {
    int par = -1;
    S.for_each(k, [&](int i) {
      if (par < 0) par = i;
    });
    if (par >= 0) {
      parent[k] = par;
      uint64_t *rp = S.row(par);
      const uint64_t *rk = S.row(k);
      for (int q = 0; q < S.words; q++) rp[q] |= rk[q];
      S.reset(par, par);
    }
  }
  return S;
}

// elimination-tree height and number of off-diagonal factor blocks of an order
std::pair<int, int64_t> etree_shape(int m, const BitRows &adj, const std::vector<int32_t> &order) {
  std::vector<int> parent;
  const BitRows S = symbolic_fill(m, adj, order, parent);
  std::vector<int> h(m, 0);
  int64_t nnz = 0;
  int height = m ? 1 : 0;
  for (int k = 0; k < m; k++) {
    nnz += S.count(k);
    if (parent[k] >= 0) {
      h[parent[k]] = std::max(h[parent[k]], h[k] + 1);
      height = std::max(height, h[parent[k]] + 1);
    }
  }
  return {height, nnz};
}

}  // namespace

// Static list schedule of the dataflow items onto kLltWaves waves. Item
// dependencies are the blocks it reads (DIAG(k): L_kp; OFF(i,k): W_k, L_ip,
// L_kp); priority is the upward rank (longest cost path to the end) with a
// rough cycle cost per item. Items are handed out in decreasing priority
// among ready ones to the wave that frees first. Each wave runs its items in
// assignment order; since every dependency was assigned earlier, the
// unfinished item with the lowest assignment index can always run (no
// deadlock), whatever the real timings.
// Item costs in shader cycles, calibrated on MI355X with tools/llt_items.py
// (N = 32 and 256): DIAG publishes L_kk / W_k after ~3.5k cycles plus its
// updates, then spends the forward step y_k on the same wave; a dependency
// hop (LDS flag, poll, s_sleep) costs a few hundred cycles.
constexpr double kCostDiag0 = 3500.0, kCostOff0 = 900.0, kCostUpd = 250.0;
constexpr double kCostPart0 = 150.0, kCostPartUpd = 60.0, kCostPartIn = 120.0;
constexpr double kCostFwd0 = 1000.0, kCostFwdUpd = 200.0, kHop = 400.0;
#ifndef M3S_SCHED_DIAG_EARLY
#define M3S_SCHED_DIAG_EARLY 1
#endif
constexpr bool kDiagEarly = M3S_SCHED_DIAG_EARLY != 0;  // (A/B: -DM3S_SCHED_DIAG_EARLY=0)
constexpr double kSlack = 300.0;  // start-time tolerance of the rank choice (small plans)

static void schedule_items(SparsePlan &P) {
  const int n = (int)P.items.size();
  const int T = (int)P.task_dst.size();
  std::vector<int> item_of_slot(P.S, -1), item_of_part(P.part_q0.size(), -1);
  for (int it = 0; it < n; it++) {
    const int v = P.items[it];
    if (v >= T) item_of_part[v - T] = it;
    else item_of_slot[v < 0 ? -1 - v : P.task_dst[v]] = it;
  }
  std::vector<std::vector<int>> deps(n), succ(n);
  std::vector<double> cost(n), pub(n);  // wave busy time; time to publishing its block
  const bool split = !P.dpart_ptr.empty();
  for (int it = 0; it < n; it++) {
    const int v = P.items[it];
    std::vector<int> &d = deps[it];
    if (v >= T) {  // PART: the blocks of its update range (+ y_p for DIAG targets)
      const int pi = v - T, tg = P.part_tgt[pi];
      for (int q = P.part_q0[pi]; q < P.part_q1[pi]; q++) {
        if (tg < 0) {
          d.push_back(item_of_slot[P.dtr_slot[q]]);
          d.push_back(item_of_slot[P.dtr_p[q]]);
        } else {
          d.push_back(item_of_slot[P.tr_a[q]]);
          d.push_back(item_of_slot[P.tr_b[q]]);
        }
      }
      cost[it] = pub[it] = kCostPart0 + kCostPartUpd * (P.part_q1[pi] - P.part_q0[pi]);
    } else if (v < 0) {
      const int k = -1 - v;
      int q0 = P.dtr_ptr[k];
      if (split) {
        for (int pi = P.dpart_ptr[k]; pi < P.dpart_ptr[k + 1]; pi++) d.push_back(item_of_part[pi]), q0 = P.part_q1[pi];
      }
      for (int q = q0; q < P.dtr_ptr[k + 1]; q++) d.push_back(item_of_slot[P.dtr_slot[q]]);
      const int nu = P.dtr_ptr[k + 1] - q0;
      const double np = split ? (double)(P.dpart_ptr[k + 1] - P.dpart_ptr[k]) : 0.0;
      pub[it] = kCostDiag0 + kCostUpd * nu + kCostPartIn * np;
      cost[it] = pub[it] + kCostFwd0 + kCostFwdUpd * nu;  // + the forward step y_k
    } else {
      d.push_back(item_of_slot[P.task_col[v]]);
      int q0 = P.task_tr_ptr[v];
      if (split) {
        for (int pi = P.opart_ptr[v]; pi < P.opart_ptr[v + 1]; pi++) d.push_back(item_of_part[pi]), q0 = P.part_q1[pi];
      }
      for (int q = q0; q < P.task_tr_ptr[v + 1]; q++) d.push_back(item_of_slot[P.tr_a[q]]);
      cost[it] = pub[it] = kCostOff0 + kCostUpd * (P.task_tr_ptr[v + 1] - q0) +
                           (split ? kCostPartIn * (P.opart_ptr[v + 1] - P.opart_ptr[v]) : 0.0);
    }
    std::sort(d.begin(), d.end());
    d.erase(std::unique(d.begin(), d.end()), d.end());
    for (int x : d) succ[x].push_back(it);
  }
  // upward rank: items are listed in a topological order (level order)
  std::vector<double> rank(n, 0.0);
  for (int it = n - 1; it >= 0; it--) {
    double best = 0.0;
    for (int s2 : succ[it]) best = std::max(best, rank[s2]);
    rank[it] = pub[it] + kHop + best;
  }
  std::vector<int> missing(n);
  std::vector<double> ready_at(n, 0.0);
  // DIAG items may start before their last input lands: the kernel's DIAG
  // sums its update products as they arrive, so a wave that takes it when all
  // but the last input are out has only the last product left when it lands
  // (round 4: C3's DIAG items were picked up after all their inputs and then
  // summed ~10 products, 1-4k cycles, on the critical path). ready_2nd: the
  // second-latest input's publish time.
  std::vector<double> ready_2nd(n, 0.0);
  using Entry = std::pair<double, int>;  // (priority, -item) max-heap
  std::priority_queue<Entry> ready;
  for (int it = 0; it < n; it++) {
    missing[it] = (int)deps[it].size();
    if (!missing[it]) ready.push({rank[it], -it});
  }
  // Simulated list scheduling onto the kernel's waves; the order in which
  // items are started is the dispatch order. The kernel's waves take items
  // from that list dynamically (an LDS counter), so a wave never idles behind
  // a mispredicted cost while ready work waits in another wave's queue. The
  // list is topological: every dependency of item i is dispatched before i,
  // so the lowest unfinished dispatched item can always run (progress).
  // Small plans (the one-workgroup LDS kernel): the free wave takes the item
  // that can START first (its inputs' predicted publish times), the highest
  // rank among those within kSlack of it. Taking the top-rank item instead
  // parked waves on items whose inputs were far off while ready work queued
  // behind them in the list (C3: one OFF item waited ~14k cycles for a wave;
  // profiles/r03/llt_stamps_r3k.txt). Large plans keep the rank heap.
  std::vector<double> free_at(kLltWaves, 0.0);
  P.witems.clear();
  std::vector<int> cand;  // ready candidates (small plans)
  std::vector<double> pub_at(n, 0.0);  // simulated publish time of each item
  const bool est_first = n <= 1024;
  if (est_first)
    while (!ready.empty()) cand.push_back(-ready.top().second), ready.pop();
  while (est_first ? !cand.empty() : !ready.empty()) {
    int w = 0;
    for (int x = 1; x < kLltWaves; x++)
      if (free_at[x] < free_at[w]) w = x;
    int it;
    if (est_first) {
      double best_est = 1e300;
      auto est = [&](int c) { return std::max(free_at[w], kDiagEarly && P.items[c] < 0 ? ready_2nd[c] : ready_at[c]); };
      for (int c : cand) best_est = std::min(best_est, est(c));
      int bi = -1;
      for (int q = 0; q < (int)cand.size(); q++) {
        const int c = cand[q];
        if (est(c) > best_est + kSlack) continue;
        if (bi < 0 || rank[c] > rank[cand[bi]] || (rank[c] == rank[cand[bi]] && c < cand[bi])) bi = q;
      }
      it = cand[bi];
      cand[bi] = cand.back();
      cand.pop_back();
    } else {
      it = -ready.top().second;
      ready.pop();
    }
    const bool early = est_first && kDiagEarly && P.items[it] < 0;
    const double start = std::max(free_at[w], early ? ready_2nd[it] : ready_at[it]);
    // an early DIAG: the products of the inputs out by `start` run first, the
    // last input's product and the factor after it lands
    const double fin = early ? std::max(start + pub[it], ready_at[it] + kCostUpd + kCostDiag0) : start + pub[it];
    free_at[w] = fin + (cost[it] - pub[it]);
    const double published = fin + kHop;
    pub_at[it] = published;
    P.witems.push_back(P.items[it]);
    for (int s2 : succ[it]) {
      if (published > ready_at[s2]) ready_2nd[s2] = ready_at[s2], ready_at[s2] = published;
      else ready_2nd[s2] = std::max(ready_2nd[s2], published);
      if (--missing[s2] == 0) {
        if (est_first) cand.push_back(s2);
        else ready.push({rank[s2], -s2});
      }
    }
  }
  // wave_ptr = {0, n}: one dispatch list shared by all waves
  P.wave_ptr.assign(1, 0);
  P.wave_ptr.push_back((int32_t)P.witems.size());
  if (split || !est_first) return;
  // Update lists of the dataflow items in the order their blocks are expected
  // to be published: the kernel applies the updates of a list as they arrive,
  // in list order, so the block that lands last should be the last product
  // (ascending p put it anywhere; what followed it waited for it). Dense-tail
  // lists keep ascending p (their border prefixes, clq's bend, rely on it).
  // Invariant: only sparse_llt_kernel (the one-workgroup factor) ever reads a
  // reordered list. Split plans (PART items: the staged global factor) return
  // above, and chip-wide plans (df_factor / column tasks / tail / column back-
  // substitution, border_kernel) are built with schedule = false and never
  // pass through here, so they keep ascending p. The reorder changes only the
  // fp64 summation order of an update sum, never its terms
  // (tests/test_sparse_plan.py solves every scheduled plan against a dense
  // fp64 solve of the same system).
  const int c0 = P.m - P.nc;
  std::vector<int> idx;
  auto reorder = [&](int q0, int q1, auto key, std::initializer_list<std::vector<int32_t> *> arrs) {
    idx.resize(q1 - q0);
    for (int q = q0; q < q1; q++) idx[q - q0] = q;
    std::stable_sort(idx.begin(), idx.end(), [&](int x, int y) { return key(x) < key(y); });
    for (std::vector<int32_t> *a : arrs) {
      std::vector<int32_t> tmp(q1 - q0);
      for (int q = q0; q < q1; q++) tmp[q - q0] = (*a)[idx[q - q0]];
      std::copy(tmp.begin(), tmp.end(), a->begin() + q0);
    }
  };
  for (int k = 0; k < c0; k++)
    reorder(P.dtr_ptr[k], P.dtr_ptr[k + 1], [&](int q) { return pub_at[item_of_slot[P.dtr_slot[q]]]; },
            {&P.dtr_slot, &P.dtr_p});
  for (int t = 0; t < T; t++)
    if (P.task_col[t] < c0)
      reorder(P.task_tr_ptr[t], P.task_tr_ptr[t + 1],
              [&](int q) { return std::max(pub_at[item_of_slot[P.tr_a[q]]], pub_at[item_of_slot[P.tr_b[q]]]); },
              {&P.tr_a, &P.tr_b});
}

void schedule_plan_items(SparsePlan &P) { schedule_items(P); }

void build_sparse_plan(int N, const std::vector<int32_t> &ri, const std::vector<int32_t> &rj,
                       SparsePlan &P, int split, int64_t max_parts, int dense_min, bool schedule) {
  const int m = N > 1 ? N - 1 : 0;
  const int64_t E = (int64_t)ri.size();
  P = SparsePlan();
  P.m = m;
  BitRows adj(m);
  for (int64_t e = 0; e < E; e++) {
    const int a = ri[e] - 1, b = rj[e] - 1;
    if (a >= 0 && b >= 0 && a != b) adj.set(a, b), adj.set(b, a);
  }
  {  // the shallowest elimination tree among MD / MMD variants (fill breaks ties)
    // The three candidates are independent: large graphs order them on three
    // threads (the plan is on a cold call's critical path; same result).
    std::vector<int32_t> o[3];
    std::pair<int, int64_t> sh[3];
    auto cand = [&](int c) {
      o[c] = min_degree_order(m, adj, c > 0, c > 0 ? c - 1 : 0);
      sh[c] = etree_shape(m, adj, o[c]);
    };
    if (m >= 96) {
      std::thread t1(cand, 1), t2(cand, 2);
      cand(0);
      t1.join();
      t2.join();
    } else {
      for (int c = 0; c < 3; c++) cand(c);
    }
    int b = 0;
    for (int c = 1; c < 3; c++)
      if (sh[c].first < sh[b].first || (sh[c].first == sh[b].first && sh[c].second < sh[b].second)) b = c;
    P.perm = std::move(o[b]);
  }
  P.iperm.assign(m, 0);
  for (int k = 0; k < m; k++) P.iperm[P.perm[k]] = k;

  // symbolic factorisation in the new order
  std::vector<int> parent;
  const BitRows Sb = symbolic_fill(m, adj, P.perm, parent);
  std::vector<std::vector<int>> st(m);
  for (int k = 0; k < m; k++) Sb.for_each(k, [&](int i) { st[k].push_back(i); });
  // slots: diagonals 0..m-1, then off-diagonals column by column
  std::vector<int32_t> slot((size_t)m * m, -1);  // slot of (i, k), i > k
  int next = m;
  P.col_ptr.assign(1, 0);
  for (int k = 0; k < m; k++) {
    for (int i : st[k]) {
      P.col_row.push_back(i);
      P.col_slot.push_back(next);
      slot[(size_t)i * m + k] = next++;
    }
    P.col_ptr.push_back((int32_t)P.col_row.size());
  }
  P.S = next;
  auto sl = [&](int i, int k) { return slot[(size_t)i * m + k]; };

  // elimination-tree levels (children before parents)
  std::vector<int> lev(m, 0);
  for (int k = 0; k < m; k++)
    if (parent[k] >= 0) lev[parent[k]] = std::max(lev[parent[k]], lev[k] + 1);
  P.levels = m ? *std::max_element(lev.begin(), lev.end()) + 1 : 0;
  P.lev_ptr.assign(P.levels + 1, 0);
  for (int k = 0; k < m; k++) P.lev_ptr[lev[k] + 1]++;
  for (int l = 0; l < P.levels; l++) P.lev_ptr[l + 1] += P.lev_ptr[l];
  P.lev_col.assign(m, 0);
  {
    std::vector<int> fill(P.lev_ptr.begin(), P.lev_ptr.end() - 1);
    for (int k = 0; k < m; k++) P.lev_col[fill[lev[k]]++] = k;
  }
  // row structure: rowst[k] = {p < k : k in struct(p)} (ascending), also as
  // bit rows R (R[k] has bit p): the update list of block (i, k) is
  // rowst[k] & rowst[i], one word-wide AND per 64 columns
  std::vector<std::vector<int>> rowst(m);
  BitRows R(m);
  for (int p = 0; p < m; p++)
    for (int i : st[p]) rowst[i].push_back(p), R.set(i, p);
  // dense tail: trailing columns whose structure is every later column
  int nc = 0;
  while (nc < m && (int)st[m - 1 - nc].size() == nc) nc++;
  if (dense_min <= 0 || nc < dense_min) nc = 0;
  const int c0 = m - nc;
  P.nc = nc;
  // left-looking updates
  P.dtr_ptr.assign(1, 0);
  for (int k = 0; k < m; k++) {
    for (int p : rowst[k]) {
      P.dtr_slot.push_back(sl(k, p));
      P.dtr_p.push_back(p);
    }
    P.dtr_ptr.push_back((int32_t)P.dtr_slot.size());
  }
  P.task_lev_ptr.assign(1, 0);
  P.ctask_ptr.assign(1, 0);
  std::vector<int32_t> ct0(nc, 0), bend((size_t)nc * nc, 0);
  for (int ci = 0; ci < nc; ci++) {  // DIAG border prefixes (dtr_p ascending)
    const int k = c0 + ci;
    int q = P.dtr_ptr[k];
    while (q < P.dtr_ptr[k + 1] && P.dtr_p[q] < c0) q++;
    bend[(size_t)ci * nc + ci] = q;
  }
  // OFF tasks in level order and their update lists, written by index into
  // arrays sized by a counting pass (push_back growth was most of this loop)
  const uint64_t *Rw = R.w.data();
  const int RW = R.words;
  auto n_common = [&](int i, int k) {
    int c = 0;
    for (int q = 0; q < RW; q++) c += __builtin_popcountll(Rw[(size_t)k * RW + q] & Rw[(size_t)i * RW + q]);
    return c;
  };
  size_t n_task = 0, n_tr = 0, n_it = 0;
  for (int k = 0; k < m; k++) {
    n_task += st[k].size();
    if (k < c0) n_it += 1 + st[k].size();
    for (int i : st[k]) n_tr += (size_t)n_common(i, k);
  }
  P.task_dst.resize(n_task);
  P.task_col.resize(n_task);
  P.task_tr_ptr.resize(n_task + 1);
  P.tr_a.resize(n_tr);
  P.tr_b.resize(n_tr);
  P.items.resize(n_it);
  P.ctask_ptr.resize((size_t)m + 1);
  P.task_lev_ptr.resize((size_t)P.levels + 1);
  int32_t *td = P.task_dst.data(), *tc = P.task_col.data(), *tp = P.task_tr_ptr.data(), *ta = P.tr_a.data(),
          *tb = P.tr_b.data(), *itm = P.items.data();
  size_t nt = 0, nr = 0, ni = 0, nct = 1;
  tp[0] = 0;
  for (int l = 0; l < P.levels; l++) {
    for (int t = P.lev_ptr[l]; t < P.lev_ptr[l + 1]; t++) {
      const int k = P.lev_col[t];
      P.ctask_ptr[nct] = P.ctask_ptr[nct - 1] + (int32_t)st[k].size();
      nct++;
      if (k < c0) {  // dense-tail columns are not dataflow items
        itm[ni++] = -1 - k;
        for (size_t q = 0; q < st[k].size(); q++) itm[ni++] = (int32_t)(nt + q);
      } else {
        ct0[k - c0] = (int32_t)nt;
      }
      const uint64_t *rk = Rw + (size_t)k * RW;
      const int32_t *slk = slot.data() + (size_t)k * m;
      for (int i : st[k]) {
        const int32_t *sli = slot.data() + (size_t)i * m;
        td[nt] = sli[k];
        tc[nt] = k;
        // p < k with i and k both in struct(p), ascending
        const uint64_t *ri_ = Rw + (size_t)i * RW;
        int32_t *bd = k >= c0 ? &bend[(size_t)(k - c0) * nc + (i - c0)] : nullptr;
        for (int q = 0; q < RW; q++)
          for (uint64_t v = rk[q] & ri_[q]; v; v &= v - 1) {
            const int p = q * 64 + __builtin_ctzll(v);
            if (bd && p < c0) *bd = (int32_t)nr + 1;
            ta[nr] = sli[p];
            tb[nr] = slk[p];
            nr++;
          }
        if (bd && *bd == 0) *bd = tp[nt];  // no border updates
        tp[++nt] = (int32_t)nr;
      }
    }
    P.task_lev_ptr[l + 1] = (int32_t)nt;
  }
  // column tasks: sparse columns in level order; first OFF task per column
  P.ctask0.assign(m, 0);
  for (int pos = 0; pos < m; pos++) {
    const int k = P.lev_col[pos];
    P.ctask0[k] = P.ctask_ptr[pos];
    if (k < c0) P.corder.push_back(k);
  }
  // the kernel addresses tail blocks arithmetically: off-diagonal slots of
  // the tail columns are the last nc (nc - 1) / 2 slots, column-major
  for (int ci = 0; ci < nc; ci++)
    for (int ri = ci + 1; ri < nc; ri++)
      if (P.task_dst[ct0[ci] + ri - ci - 1] != P.S - nc * (nc - 1) / 2 + ci * nc - ci * (ci + 1) / 2 + ri - ci - 1)
        nc = -1;  // not contiguous (never expected): no dense tail
  if (nc < 0) return build_sparse_plan(N, ri, rj, P, split, max_parts, 0, schedule);
  P.clq.assign(1, nc);
  P.clq.push_back(c0);
  P.clq.insert(P.clq.end(), ct0.begin(), ct0.end());
  P.clq.insert(P.clq.end(), bend.begin(), bend.end());
  if (split > 0) {
    // count parts first; widen the split until they fit the buffer
    auto n_parts = [&](int sp) {
      int64_t c = 0;
      for (int k = 0; k < c0; k++) c += std::max(0, (P.dtr_ptr[k + 1] - P.dtr_ptr[k] - 1) / sp);
      for (size_t t = 0; t < P.task_dst.size(); t++)
        if (P.task_col[t] < c0) c += std::max(0, (P.task_tr_ptr[t + 1] - P.task_tr_ptr[t] - 1) / sp);
      return c;
    };
    while (n_parts(split) > max_parts) split *= 2;
    // items again, column by column: the parts of DIAG(k) and of OFF(., k)
    // (inputs from earlier columns only) precede DIAG(k)
    const int T = (int)P.task_dst.size();
    std::vector<int32_t> items;
    P.dpart_ptr.assign(m + 1, 0);
    P.opart_ptr.assign(T + 1, 0);
    std::vector<std::vector<int32_t>> dparts(m), oparts(T);
    auto add_parts = [&](int tgt, int q0, int q1, std::vector<int32_t> &out) {
      const int np = std::max(0, (q1 - q0 - 1) / split);
      for (int j = 0; j < np; j++) {
        out.push_back((int32_t)P.part_q0.size());
        P.part_q0.push_back(q0 + j * split);
        P.part_q1.push_back(q0 + (j + 1) * split);
        P.part_tgt.push_back(tgt);
      }
    };
    // part indices are assigned target by target (DIAG targets in column
    // order, then OFF tasks in task order) so each target's parts are contiguous
    for (int k = 0; k < c0; k++) add_parts(-1 - k, P.dtr_ptr[k], P.dtr_ptr[k + 1], dparts[k]);
    for (int t = 0; t < T; t++)
      if (P.task_col[t] < c0) add_parts(t, P.task_tr_ptr[t], P.task_tr_ptr[t + 1], oparts[t]);
    for (int k = 0; k < m; k++) P.dpart_ptr[k + 1] = P.dpart_ptr[k] + (int32_t)dparts[k].size();
    P.opart_ptr[0] = P.dpart_ptr[m];  // OFF parts follow the DIAG parts
    for (int t = 0; t < T; t++) P.opart_ptr[t + 1] = P.opart_ptr[t] + (int32_t)oparts[t].size();
    int t = 0;
    for (int l = 0; l < P.levels; l++)
      for (int pos = P.lev_ptr[l]; pos < P.lev_ptr[l + 1]; pos++) {
        const int k = P.lev_col[pos];
        if (k >= c0) {  // dense tail
          t += (int)st[k].size();
          continue;
        }
        for (int32_t pi : dparts[k]) items.push_back(T + pi);
        for (int q = 0; q < (int)st[k].size(); q++)
          for (int32_t pi : oparts[t + q]) items.push_back(T + pi);
        items.push_back(-1 - k);
        for (int q = 0; q < (int)st[k].size(); q++) items.push_back(t + q);
        t += (int)st[k].size();
      }
    P.items.swap(items);
  }
  if (schedule) schedule_items(P);
  // assembly lists (edge order => deterministic sums), by counting sort
  P.asm_ptr.assign(P.S + 1, 0);
  P.g_ptr.assign(m + 1, 0);
  auto ends = [&](int64_t e, int &pa, int &pb) {
    const int a = ri[e] - 1, b = rj[e] - 1;
    pa = a >= 0 ? P.iperm[a] : -1, pb = b >= 0 ? P.iperm[b] : -1;
    return a != b;  // Hs[0]+Hs[1]+Hs[2]+Hs[3] = 0 on the same pose
  };
  for (int64_t e = 0; e < E; e++) {
    int pa, pb;
    if (!ends(e, pa, pb)) continue;
    if (pa >= 0) P.asm_ptr[pa + 1]++, P.g_ptr[pa + 1]++;
    if (pb >= 0) P.asm_ptr[pb + 1]++, P.g_ptr[pb + 1]++;
    if (pa >= 0 && pb >= 0) P.asm_ptr[sl(std::max(pa, pb), std::min(pa, pb)) + 1]++;
  }
  for (int q = 0; q < P.S; q++) P.asm_ptr[q + 1] += P.asm_ptr[q];
  for (int q = 0; q < m; q++) P.g_ptr[q + 1] += P.g_ptr[q];
  P.asm_edge.assign(P.asm_ptr[P.S], 0);
  P.g_edge.assign(P.g_ptr[m], 0);
  std::vector<int32_t> af(P.asm_ptr.begin(), P.asm_ptr.end() - 1), gf(P.g_ptr.begin(), P.g_ptr.end() - 1);
  for (int64_t e = 0; e < E; e++) {
    int pa, pb;
    if (!ends(e, pa, pb)) continue;
    if (pa >= 0) P.asm_edge[af[pa]++] = (int32_t)e, P.g_edge[gf[pa]++] = (int32_t)(e << 1);
    if (pb >= 0) P.asm_edge[af[pb]++] = (int32_t)e, P.g_edge[gf[pb]++] = (int32_t)(e << 1 | 1);
    if (pa >= 0 && pb >= 0) {
      const int s2 = sl(std::max(pa, pb), std::min(pa, pb));
      P.asm_edge[af[s2]++] = (int32_t)e;
    }
  }
}

void flatten_plan(const SparsePlan &P, PlanImage &img) {
  img.data.clear();
  auto put = [&](const std::vector<int32_t> &v) {
    const int64_t off = (int64_t)img.data.size();
    img.data.insert(img.data.end(), v.begin(), v.end());
    while (img.data.size() % 4) img.data.push_back(0);  // 16-B aligned sections
    return off;
  };
  img.off_perm = put(P.perm);
  img.off_col_ptr = put(P.col_ptr);
  img.off_col_row = put(P.col_row);
  img.off_col_slot = put(P.col_slot);
  img.off_lev_ptr = put(P.lev_ptr);
  img.off_lev_col = put(P.lev_col);
  img.off_dtr_ptr = put(P.dtr_ptr);
  img.off_dtr_slot = put(P.dtr_slot);
  img.off_dtr_p = put(P.dtr_p);
  img.off_task_lev_ptr = put(P.task_lev_ptr);
  img.off_task_dst = put(P.task_dst);
  img.off_task_col = put(P.task_col);
  img.off_task_tr_ptr = put(P.task_tr_ptr);
  img.off_tr_a = put(P.tr_a);
  img.off_tr_b = put(P.tr_b);
  img.off_asm_ptr = put(P.asm_ptr);
  img.off_asm_edge = put(P.asm_edge);
  img.off_g_ptr = put(P.g_ptr);
  img.off_g_edge = put(P.g_edge);
  img.off_ctask_ptr = put(P.ctask_ptr);
  img.off_items = put(P.items);
  img.off_wave_ptr = put(P.wave_ptr);
  img.off_witems = put(P.witems);
  img.off_part_q0 = put(P.part_q0);
  img.off_part_q1 = put(P.part_q1);
  img.off_part_tgt = put(P.part_tgt);
  img.off_dpart_ptr = put(P.dpart_ptr);
  img.off_opart_ptr = put(P.opart_ptr);
  img.off_clq = put(P.clq);
  img.off_corder = put(P.corder);
  img.off_ctask0 = put(P.ctask0);
}

}  // namespace m3s
