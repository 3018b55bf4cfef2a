// m3s_symbolic.h — host-side symbolic analysis for the block-sparse LLT.
//
// The reference solves the (N-1)*7 pose system with Eigen's SimplicialLLT
// (gn_kernels.cu:132-153), i.e. a sparse Cholesky behind a fill-reducing
// ordering. This is the same idea with 7x7 blocks: one variable per free pose,
// a minimum-degree ordering, the block fill pattern, and a level schedule of
// the elimination tree so the numeric phase (m3s_gn.hip, sparse_llt_kernel)
// can factor independent columns concurrently. Computed once per solve call
// (the edge structure is fixed across its GN iterations).
#pragma once
#include <stdint.h>

#include <vector>

namespace m3s {

struct SparsePlan {
  int m = 0;       // free poses (N - 1)
  int S = 0;       // 7x7 block slots of L: [0, m) diagonals, then off-diagonals
  int levels = 0;  // elimination-tree levels
  std::vector<int32_t> perm;   // new -> old variable
  std::vector<int32_t> iperm;  // old -> new
  // per column k (new order): struct(k) = rows i > k with L_ik != 0
  std::vector<int32_t> col_ptr, col_row, col_slot;
  // columns grouped by level (leaves first)
  std::vector<int32_t> lev_ptr, lev_col;
  // left-looking diagonal updates of column k: D_k -= L_kp L_kp^T
  std::vector<int32_t> dtr_ptr, dtr_slot, dtr_p;
  // off-diagonal tasks (one output block L_ik each), grouped by level
  std::vector<int32_t> task_lev_ptr, task_dst, task_col, task_tr_ptr, tr_a, tr_b;
  // assembly: slot s receives sum over asm edges of (+H_jj diag, -H_jj off-diag)
  std::vector<int32_t> asm_ptr, asm_edge;
  // RHS of new variable v: sum over entries (edge << 1 | sign) of (sign ? +g_j : -g_j)
  std::vector<int32_t> g_ptr, g_edge;
  // off-diagonal tasks of the column at level-order position t: [ctask_ptr[t], ctask_ptr[t+1])
  std::vector<int32_t> ctask_ptr;
  // dataflow work items in level order: -1-k = DIAG(k), t >= 0 = off-diagonal task t
  std::vector<int32_t> items;
  // Split updates (large factors): the head of a long update list runs as
  // PART items (item code T + part index) that sum up to `split` products into
  // a partial block as soon as their inputs exist; the DIAG / OFF item then
  // adds the partials in part order and does only its tail. Part p covers
  // update entries [part_q0[p], part_q1[p]) of its target (dtr list for
  // DIAG(k) targets, tr list for OFF(t)); target code -1-k or t.
  std::vector<int32_t> part_q0, part_q1, part_tgt;
  std::vector<int32_t> dpart_ptr, opart_ptr;  // parts of DIAG(k) / OFF(t), contiguous
  // dispatch order of the items (host list scheduling by upward rank; a
  // topological order): the kernel's waves take witems[0 .. wave_ptr[1]) in
  // this order from a shared counter
  std::vector<int32_t> wave_ptr, witems;
  // Dense tail: the trailing nc columns whose structure is every later column
  // (the top of the elimination tree is a dense clique) are not dataflow
  // items; sparse_llt_kernel factors them after the items, bulk-synchronously
  // and right-looking. clq = {nc, c0 = m - nc, ct0[nc], bend[nc * nc]}:
  // ct0[ci] = first OFF task of column c0 + ci (task of row c0 + ri is
  // ct0[ci] + ri - ci - 1); bend[ci * nc + ri] = end of the border prefix
  // (updates from columns p < c0) of the target (c0 + ri, c0 + ci) in its
  // update list (dtr list for ri == ci, tr list otherwise). nc = 0: none.
  int nc = 0;
  std::vector<int32_t> clq;
  // Column tasks (multi-workgroup factorisation, col_factor_kernel): the
  // sparse columns (< m - nc) in level order (a topological order), and the
  // first OFF task of every column (its |struct(k)| tasks are contiguous).
  std::vector<int32_t> corder, ctask0;
};

// ranks of (ii, jj) in sorted-unique(cat(ii, jj)); returns the unique count
int host_remap(const int64_t *ii, const int64_t *jj, int64_t E, std::vector<int32_t> &ri,
               std::vector<int32_t> &rj);

// Build the plan for N poses (rank 0 fixed) and edges with ranks (ri, rj).
// split > 0 enables PART items of `split` updates each (at most max_parts).
// dense_min: smallest top clique handled as a dense tail (0: never)
constexpr int kDenseTailMin = 16;  // measured (ab_dense_tail_min.txt): a win at 42 (N = 256) and at 18 (N = 128, factor + back-sub 339 -> 253 us), a loss at 10 (N = 64)
// schedule = false leaves wave_ptr / witems empty (only sparse_llt_kernel, the
// one-workgroup factor, reads them; schedule_plan_items fills them later)
void build_sparse_plan(int N, const std::vector<int32_t> &ri, const std::vector<int32_t> &rj,
                       SparsePlan &P, int split = 0, int64_t max_parts = 0, int dense_min = kDenseTailMin,
                       bool schedule = true);
void schedule_plan_items(SparsePlan &P);

// Flattened int32 image of the plan (offsets of each array into it).
struct PlanImage {
  std::vector<int32_t> data;
  int64_t off_perm, off_col_ptr, off_col_row, off_col_slot, off_lev_ptr, off_lev_col, off_dtr_ptr,
      off_dtr_slot, off_dtr_p, off_task_lev_ptr, off_task_dst, off_task_col, off_task_tr_ptr,
      off_tr_a, off_tr_b, off_asm_ptr, off_asm_edge, off_g_ptr, off_g_edge, off_ctask_ptr,
      off_items, off_wave_ptr, off_witems, off_part_q0, off_part_q1, off_part_tgt, off_dpart_ptr,
      off_opart_ptr, off_clq, off_corder, off_ctask0;
};
constexpr int kPlanSections = 31;
constexpr int kLltWaves = 16;  // waves of sparse_llt_kernel (1024 threads)
void flatten_plan(const SparsePlan &P, PlanImage &img);

}  // namespace m3s
