// Host-side structure analysis for one ba() call (the part of ba_cuda that
// depends only on ii, jj, t0, t1): droid_kernels.cu:1336-1345 (ts, kx, kk),
// :1241-1272 (Schur row graph) and the triplet lists of
// SparseBlock::update_lhs/rhs (:1131-1173).  Unlike the reference, this runs
// once per edge set (cached by the caller), never inside the GN loop.
#include <algorithm>
#include <cstring>
#include <functional>
#include <map>
#include <queue>
#include <tuple>
#include <utility>

#include "ba.hpp"
#include "common.hpp"

namespace droid {

static size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Task DAG of the dataflow Cholesky (ba_kernels.hip: chol_dataflow_kernel) for
// the augmented system with n pivots and the rhs as row n:
//   POTRF(k)     factor tile (k,k) (+ the rhs row when it lies in that tile), Linv_k
//   TRSM(i,k)    tile (i,k) <- A_ik Linv_k^T
//   UPD(i,j,k)   tile (i,j) -= L_ik L_jk^T               (k < j <= i)
//   BSOLVE(c)    x_c = Linv_c^T y_c
//   BUPD(r,c)    y_c -= L_rc^T x_r                       (c < r, applied in order r = nbc-1 .. c+1)
// Tickets are handed out in a list-scheduling order: among ready tasks, the
// longest remaining path (estimated microseconds incl. one hop per edge) first.
void build_chol_tasks(int n, int& nbc, int& nbr, std::vector<int>& out) {
  nbc = (n + 63) / 64;
  nbr = (n + 1 + 63) / 64;
  out.clear();
  if (n <= 0) return;
  struct Node { int type, i, j, k; double cost; std::vector<int> succ; int npred; double bl; };
  std::vector<Node> t;
  std::map<std::tuple<int, int, int, int>, int> id;
  auto add = [&](int type, int i, int j, int k, double cost) {
    id[std::make_tuple(type, i, j, k)] = (int)t.size();
    t.push_back({type, i, j, k, cost, {}, 0, 0.0});
  };
  // potrf(k) also applies the last update of its own tile, (k,k,k-1), and
  // solves the tile below it, trsm(k+1,k): the diagonal chain hands off once
  // per step instead of three times.
  for (int k = 0; k < nbc; ++k) {
    add(kPotrf, k, k, k, 10.0);
    for (int i = k + 2; i < nbr; ++i) add(kTrsm, i, k, k, 2.0);
    for (int j = k + 1; j < nbc; ++j)
      for (int i = j; i < nbr; ++i)
        if (!(i == j && j == k + 1)) add(kUpdate, i, j, k, 2.0);
  }
  // bsolve(c) also applies x_c to y_{c-1} (bupd(c, c-1)): one hand-off per
  // step of the back-substitution chain
  for (int c = 0; c < nbc; ++c) {
    add(kBsolve, c, c, c, 2.0);
    for (int r = c + 2; r < nbc; ++r) add(kBupd, r, c, c, 1.0);
  }
  auto get = [&](int type, int i, int j, int k) { return id.at(std::make_tuple(type, i, j, k)); };
  auto fin = [&](int i, int k) { return (i == k || i == k + 1) ? get(kPotrf, k, k, k) : get(kTrsm, i, k, k); };
  // the task that applies x_r to y_c
  auto ychain = [&](int r, int c) { return r == c + 1 ? get(kBsolve, r, r, r) : get(kBupd, r, c, c); };
  auto edge = [&](int a, int b) {
    for (int x : t[a].succ)
      if (x == b) return;
    t[a].succ.push_back(b);
    t[b].npred++;
  };
  for (int v = 0; v < (int)t.size(); ++v) {
    const Node nd = t[v];
    switch (nd.type) {
      case kPotrf:
        if (nd.k >= 2) edge(get(kUpdate, nd.k, nd.k, nd.k - 2), v);
        if (nd.k >= 1) edge(get(kPotrf, nd.k - 1, nd.k - 1, nd.k - 1), v);
        if (nd.k >= 1 && nd.k + 1 < nbr) edge(get(kUpdate, nd.k + 1, nd.k, nd.k - 1), v);
        break;
      case kTrsm:
        edge(get(kPotrf, nd.k, nd.k, nd.k), v);
        if (nd.k > 0) edge(get(kUpdate, nd.i, nd.k, nd.k - 1), v);
        break;
      case kUpdate:
        edge(fin(nd.i, nd.k), v);
        edge(fin(nd.j, nd.k), v);
        if (nd.k > 0) edge(get(kUpdate, nd.i, nd.j, nd.k - 1), v);
        break;
      case kBsolve:
        edge(get(kPotrf, nd.i, nd.i, nd.i), v);
        edge(nd.i == nbc - 1 ? fin(nbr - 1, nd.i) : ychain(nd.i + 1, nd.i), v);
        if (nd.i >= 1) {
          edge(fin(nd.i, nd.i - 1), v);
          edge(nd.i == nbc - 1 ? fin(nbr - 1, nd.i - 1) : ychain(nd.i + 1, nd.i - 1), v);
        }
        break;
      case kBupd:
        edge(get(kBsolve, nd.i, nd.i, nd.i), v);
        edge(fin(nd.i, nd.j), v);
        edge(nd.i == nbc - 1 ? fin(nbr - 1, nd.j) : ychain(nd.i + 1, nd.j), v);
        break;
    }
  }
  // bottom levels (reverse topological order)
  std::vector<int> order, indeg(t.size());
  for (size_t v = 0; v < t.size(); ++v) indeg[v] = t[v].npred;
  for (size_t v = 0; v < t.size(); ++v)
    if (!indeg[v]) order.push_back((int)v);
  for (size_t q = 0; q < order.size(); ++q)
    for (int s2 : t[order[q]].succ)
      if (--indeg[s2] == 0) order.push_back(s2);
  for (int q = (int)order.size() - 1; q >= 0; --q) {
    Node& nd = t[order[q]];
    double m = 0.0;
    for (int s2 : nd.succ) m = std::max(m, 1.0 + t[s2].bl);
    nd.bl = nd.cost + m;
  }
  // list scheduling by bottom level
  auto cmp = [&](int a, int b) { return t[a].bl != t[b].bl ? t[a].bl < t[b].bl : a > b; };
  std::priority_queue<int, std::vector<int>, decltype(cmp)> ready(cmp);
  for (size_t v = 0; v < t.size(); ++v) {
    indeg[v] = t[v].npred;
    if (!indeg[v]) ready.push((int)v);
  }
  while (!ready.empty()) {
    const int v = ready.top();
    ready.pop();
    out.push_back(t[v].type); out.push_back(t[v].i); out.push_back(t[v].j); out.push_back(t[v].k);
    for (int s2 : t[v].succ)
      if (--indeg[s2] == 0) ready.push(s2);
  }
}

static int build_plan(BaPlan& p, const int64_t* ii, const int64_t* jj, int E, int N, int H, int W,
                      int t0, int t1, int eta_rows, int motion_only, int own_lo, int own_hi) {
  if (E < 0 || N <= 0 || H <= 0 || W <= 0) return fail(kInvalidArgument, "ba: bad sizes");
  if (t0 < 0 || t1 <= t0 || t1 > N)
    return fail(kInvalidArgument, "ba: need 0 <= t0 < t1 <= num_frames");
  p.E = E; p.N = N; p.H = H; p.W = W; p.HW = H * W;
  p.t0 = t0; p.t1 = t1; p.P = t1 - t0; p.n = 6 * p.P;
  p.motion_only = motion_only; p.eta_rows = eta_rows;
  p.ii.resize(E); p.jj.resize(E);
  for (int e = 0; e < E; ++e) {
    if (ii[e] < 0 || ii[e] >= N || jj[e] < 0 || jj[e] >= N)
      return fail(kInvalidArgument, "ba: edge index out of range");
    p.ii[e] = (int)ii[e];
    p.jj[e] = (int)jj[e];
  }
  const int HW = p.HW;

  // kx = unique(cat(ts, ii)) with ts the optimised poses this rank owns
  std::vector<char> present(N, 0);
  const int lo = std::max(t0, own_lo), hi = std::min(t1, own_hi);
  for (int t = lo; t < hi; ++t) present[t] = 1;
  for (int e = 0; e < E; ++e) present[p.ii[e]] = 1;
  std::vector<int> fidx(N, -1);
  p.kx.clear();
  for (int f = 0; f < N; ++f)
    if (present[f]) { fidx[f] = (int)p.kx.size(); p.kx.push_back(f); }
  p.K = (int)p.kx.size();
  if (!motion_only && eta_rows != p.K && eta_rows != 1)
    return fail(kInvalidArgument,
                "ba: eta must have one row per frame of unique([t0,t1) U ii) (got " +
                    std::to_string(eta_rows) + ", need " + std::to_string(p.K) + ")");

  // edges grouped by source frame, ascending edge index (stable)
  p.f_eptr.assign(p.K + 1, 0);
  for (int e = 0; e < E; ++e) p.f_eptr[fidx[p.ii[e]] + 1]++;
  for (int f = 0; f < p.K; ++f) p.f_eptr[f + 1] += p.f_eptr[f];
  p.f_edges.assign(E, 0);
  {
    std::vector<int> fill(p.f_eptr.begin(), p.f_eptr.end() - 1);
    for (int e = 0; e < E; ++e) p.f_edges[fill[fidx[p.ii[e]]]++] = e;
  }

  // launch geometry
  p.nsplit = std::max(1, std::min(std::max(1, HW / 256), (2048 + std::max(E, 1) - 1) / std::max(E, 1)));
  const int rounds = ceil_div(HW, 256);
  p.group_per_wave = std::max(1, std::min(rounds, (int)((long)p.K * rounds / 1024)));
  p.nchunk = ceil_div(rounds, p.group_per_wave);

  // Schur rows per frame: [Ei row if the frame's pose is optimised] + one Eij row per edge
  p.f_rptr.assign(p.K + 1, 0);
  p.r_pose.clear(); p.r_edge.clear();
  p.f_nb.assign(p.K, 0); p.f_goff.assign(p.K, 0);
  p.nb_max = 1;
  p.gram_floats = 0;
  for (int f = 0; f < p.K; ++f) {
    const int kf = p.kx[f];
    if (kf >= t0 && kf < t1) { p.r_pose.push_back(kf - t0); p.r_edge.push_back(-1); }
    for (int k = p.f_eptr[f]; k < p.f_eptr[f + 1]; ++k) {
      const int e = p.f_edges[k];
      const int j = p.jj[e];
      p.r_pose.push_back((j >= t0 && j < t1) ? j - t0 : -1);
      p.r_edge.push_back(e);
    }
    p.f_rptr[f + 1] = (int)p.r_pose.size();
    const int nrows = p.f_rptr[f + 1] - p.f_rptr[f];
    const int nb = ceil_div(6 * nrows + 1, 16);
    if (!motion_only && nb > kNbMax)
      return fail(kUnsupported, "ba: a depth frame has " + std::to_string(nrows - 1) +
                                    " outgoing edges; the Schur kernel supports up to 20");
    p.f_nb[f] = nb;
    p.nb_max = std::max(p.nb_max, nb);
    p.f_goff[f] = (int)p.gram_floats;
    p.gram_floats += (long)p.nchunk * (nb * (nb + 1) / 2) * 256;
  }
  if (motion_only) p.gram_floats = 0;

  // Block contribution lists for the lower triangle of the reduced system.
  std::map<std::pair<int, int>, std::vector<Contrib>> blocks;
  std::vector<std::vector<Contrib>> rhs(p.P);
  const int P = p.P;
  for (int e = 0; e < E; ++e) {
    const int i = p.ii[e] - t0, j = p.jj[e] - t0;
    const int idx[2] = {i, j};
    for (int a = 0; a < 2; ++a)
      for (int b = 0; b < 2; ++b) {
        const int r = idx[a], c = idx[b];
        if (r < 0 || c < 0 || r >= P || c >= P || r < c) continue;
        blocks[{r, c}].push_back({kEdgeBlock, e, 6 * a, 6 * b});
      }
    if (i >= 0 && i < P) rhs[i].push_back({kEdgeRhs, e, 0, 0});
    if (j >= 0 && j < P) rhs[j].push_back({kEdgeRhs, e, 6, 0});
  }
  if (!motion_only) {
    for (int f = 0; f < p.K; ++f) {
      const int r0 = p.f_rptr[f], r1 = p.f_rptr[f + 1];
      for (int ra = r0; ra < r1; ++ra) {
        const int pa = p.r_pose[ra];
        if (pa < 0) continue;
        rhs[pa].push_back({kSchurRhs, f, ra - r0, 0});
        for (int rb = r0; rb < r1; ++rb) {
          const int pb = p.r_pose[rb];
          if (pb < 0 || pa < pb) continue;
          blocks[{pa, pb}].push_back({kSchurBlock, f, ra - r0, rb - r0});
        }
      }
    }
  }
  p.blk_a.clear(); p.blk_b.clear(); p.blk_cptr.assign(1, 0); p.contrib.clear();
  for (auto& kv : blocks) {
    p.blk_a.push_back(kv.first.first);
    p.blk_b.push_back(kv.first.second);
    for (auto& c : kv.second) p.contrib.push_back(c);
    p.blk_cptr.push_back((int)p.contrib.size());
  }
  p.rhs_cptr.assign(1, 0); p.rhs_contrib.clear();
  for (int a = 0; a < P; ++a) {
    for (auto& c : rhs[a]) p.rhs_contrib.push_back(c);
    p.rhs_cptr.push_back((int)p.rhs_contrib.size());
  }

  // pack the int section
  p.ints.clear();
  auto put = [&](const std::vector<int>& v) {
    size_t o = p.ints.size();
    p.ints.insert(p.ints.end(), v.begin(), v.end());
    while (p.ints.size() % 4) p.ints.push_back(0);
    return o;
  };
  auto putc = [&](const std::vector<Contrib>& v) {
    size_t o = p.ints.size();
    for (auto& c : v) { p.ints.push_back(c.kind); p.ints.push_back(c.src); p.ints.push_back(c.a0); p.ints.push_back(c.a1); }
    return o;
  };
  p.o_ii = put(p.ii); p.o_jj = put(p.jj); p.o_kx = put(p.kx);
  p.o_feptr = put(p.f_eptr); p.o_fedges = put(p.f_edges);
  p.o_frptr = put(p.f_rptr); p.o_rpose = put(p.r_pose); p.o_redge = put(p.r_edge);
  p.o_fnb = put(p.f_nb); p.o_fgoff = put(p.f_goff);
  p.o_blka = put(p.blk_a); p.o_blkb = put(p.blk_b); p.o_blkcptr = put(p.blk_cptr);
  p.o_rhscptr = put(p.rhs_cptr);
  p.o_contrib = putc(p.contrib); p.o_rhscontrib = putc(p.rhs_contrib);
  build_chol_tasks(p.n, p.nbc, p.nbr, p.tasks);
  p.ntasks = (int)p.tasks.size() / 4;
  p.o_tasks = put(p.tasks);
  if (p.ints.empty()) p.ints.push_back(0);
  p.ld = (p.n + 1 + 7) / 8 * 8;
  p.sync_bytes = align_up((size_t)(4 + p.nbr * p.nbc + 2 * p.nbc) * 4, 16);

  // workspace layout
  size_t off = 0;
  p.off_ints = off; off = align_up(off + p.ints.size() * 4, 256);
  p.off_hpart = off; off = align_up(off + (size_t)std::max(E, 1) * p.nsplit * kHessStride * 4, 256);
  p.off_gram = off; off = align_up(off + (size_t)std::max(p.gram_floats, 1L) * 4, 256);
  p.off_qw = off; off = align_up(off + (size_t)2 * p.K * HW * 4 + 4, 256);
  p.off_M = off; off = align_up(off + (size_t)(p.n + 1) * p.ld * 8, 256);
  p.off_x = off; off = align_up(off + (size_t)(p.n + 1) * 8, 256);
  p.off_flag = off; off = align_up(off + 64, 256);
  p.off_sync = off; off = align_up(off + p.sync_bytes, 256);
  p.off_linv = off; off = align_up(off + (size_t)std::max(p.nbc, 1) * 64 * 64 * 8, 256);
  p.off_ybuf = off; off = align_up(off + (size_t)std::max(p.nbc, 1) * 64 * 8, 256);
  p.total = off;
  return kOk;
}

}  // namespace droid

using namespace droid;

extern "C" {

int droid_ba_plan_create(const int64_t* ii, const int64_t* jj, int num_edges, int num_frames,
                         int ht, int wd, int t0, int t1, int eta_rows, int motion_only,
                         int own_lo, int own_hi, void** plan_out) {
  if (!plan_out) return fail(kInvalidArgument, "ba_plan_create: null output");
  *plan_out = nullptr;
  auto* p = new BaPlan();
  int st = build_plan(*p, ii, jj, num_edges, num_frames, ht, wd, t0, t1, eta_rows, motion_only,
                      own_lo, own_hi);
  if (st != kOk) { delete p; return st; }
  *plan_out = p;
  return kOk;
}

// Dense SPD solve of an augmented system on the dataflow Cholesky alone (no
// BA): n pivots, ld = n+1 rounded up to 8; rows 0..n-1 hold the lower
// triangle of A, row n the rhs b (droid_ba_plan_system_region locates it).
int droid_chol_plan_create(int n, void** plan_out) {
  if (!plan_out || n < 0) return fail(kInvalidArgument, "chol_plan_create: bad arguments");
  auto* p = new BaPlan();
  p->n = n;
  p->P = 0;
  p->motion_only = 1;
  build_chol_tasks(n, p->nbc, p->nbr, p->tasks);
  p->ntasks = (int)p->tasks.size() / 4;
  p->ints = p->tasks;
  p->o_tasks = 0;
  if (p->ints.empty()) p->ints.push_back(0);
  p->ld = (n + 1 + 7) / 8 * 8;
  p->sync_bytes = align_up((size_t)(4 + p->nbr * p->nbc + 2 * p->nbc) * 4, 16);
  size_t off = 0;
  p->off_ints = off; off = align_up(off + p->ints.size() * 4, 256);
  p->off_M = off; off = align_up(off + (size_t)(n + 1) * p->ld * 8, 256);
  p->off_x = off; off = align_up(off + (size_t)(n + 1) * 8, 256);
  p->off_flag = off; off = align_up(off + 64, 256);
  p->off_sync = off; off = align_up(off + p->sync_bytes, 256);
  p->off_linv = off; off = align_up(off + (size_t)std::max(p->nbc, 1) * 64 * 64 * 8, 256);
  p->off_ybuf = off; off = align_up(off + (size_t)std::max(p->nbc, 1) * 64 * 8, 256);
  p->total = off;
  *plan_out = p;
  return kOk;
}

int droid_chol_plan_info(const void* plan, int* ld, int* ntasks, int* flag_offset) {
  auto* p = static_cast<const BaPlan*>(plan);
  if (!p) return fail(kInvalidArgument, "chol_plan_info: null plan");
  if (ld) *ld = p->ld;
  if (ntasks) *ntasks = p->ntasks;
  if (flag_offset) *flag_offset = (int)p->off_flag;
  return kOk;
}

// the plan's Cholesky task list in ticket order (4 ints per task: type, i, j, k)
int droid_chol_plan_tasks(const void* plan, int* out) {
  auto* p = static_cast<const BaPlan*>(plan);
  if (!p || !out) return fail(kInvalidArgument, "chol_plan_tasks: null argument");
  std::copy(p->tasks.begin(), p->tasks.end(), out);
  return kOk;
}

void droid_ba_plan_destroy(void* plan) { delete static_cast<BaPlan*>(plan); }

size_t droid_ba_plan_workspace_bytes(const void* plan) {
  return plan ? static_cast<const BaPlan*>(plan)->total : 0;
}

int droid_ba_plan_info(const void* plan, int* K, int* P, int* nblocks, int* nb_max) {
  auto* p = static_cast<const BaPlan*>(plan);
  if (!p) return fail(kInvalidArgument, "ba_plan_info: null plan");
  if (K) *K = p->K;
  if (P) *P = p->P;
  if (nblocks) *nblocks = (int)p->blk_a.size();
  if (nb_max) *nb_max = p->nb_max;
  return kOk;
}

int droid_ba_plan_kx(const void* plan, int64_t* out) {
  auto* p = static_cast<const BaPlan*>(plan);
  if (!p) return fail(kInvalidArgument, "ba_plan_kx: null plan");
  for (int k = 0; k < p->K; ++k) out[k] = p->kx[k];
  return kOk;
}

// Byte offset/size of the reduced system (augmented, n+1 rows of ld fp64 with
// ld = n+1 rounded up to 8, rhs in the last row) inside the workspace: the
// buffer a multi-GPU caller all-reduces.
int droid_ba_plan_system_region(const void* plan, size_t* offset, size_t* bytes) {
  auto* p = static_cast<const BaPlan*>(plan);
  if (!p) return fail(kInvalidArgument, "ba_plan_system_region: null plan");
  *offset = p->off_M;
  *bytes = (size_t)(p->n + 1) * p->ld * 8;
  return kOk;
}

}  // extern "C"
