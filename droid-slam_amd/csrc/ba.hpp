// Dense bundle adjustment (ba_cuda, droid_kernels.cu:1314-1434) on the GPU.
//
// Host side (ba_plan.cpp) turns the edge list of one ba() call into a static
// "plan": the depth frames kx, per-frame edge lists, the rows of the Schur
// complement per frame, a deterministic contribution list for every nonzero
// 6x6 block of the reduced camera system, a fill-reducing order of the poses
// and the tile-sparse structure of the factor.  Device side (ba_kernels.hip)
// runs every Gauss-Newton iteration with no host round trip:
//
//   ba_edge_hessian      per edge: 12x12 Hessian + 12 gradient (JtWJ, JtWr)
//   ba_frame_schur<NB>   per depth frame: C, w, Q = 1/C, E rows, and the Gram
//                        [E w]^T diag(Q) [E w] on f32 MFMA (S and S-rhs at once)
//   ba_frame_prep +      the same for frames with more rows than one workgroup's
//   ba_frame_gram_wide   registers hold (no out-degree limit): Q, w, Ei first,
//                        then the Gram in 64x64 blocks, one workgroup per block
//   ba_assemble          deterministic gather of A - S into the 64x64 fp64 tiles
//                        of the permuted system, rhs as its last row
//   chol_dataflow        ONE persistent launch: tile-sparse right-looking fp64
//                        Cholesky (forward solve rides along in the appended
//                        row) and the back solve, tile tasks handed out by
//                        ticket in critical-path order and synchronised by
//                        per-tile version counters (no grid barriers)
//   ba_backsub           dz = Q (w - sum E^T dx) with the reference's t0 skip
//   ba_retract           poses <- Exp(dx) poses
//
// The reference solves the same system with Eigen's SimplicialLLT (AMD
// ordering, droid_kernels.cu:1192-1213); here the pose order is chosen at plan
// time among identity / reverse Cuthill-McKee / minimum degree by the number of
// tile tasks it leaves, and only structurally nonzero 64x64 tiles of the factor
// are stored, reduced over ranks and factored.
#pragma once
#include <stdint.h>
#include <vector>

namespace droid {

constexpr int kHessVals = 90;      // 78 upper-tri of 12x12 + 6 vi + 6 vj
constexpr int kHessStride = 96;    // padded per (edge, split)
constexpr int kCholBlock = 64;
constexpr int kTile = 64 * 64;     // doubles per stored tile
constexpr int kNbMax = 8;          // Gram tiles per side in registers: 16*8 = 128 vars -> 21 rows/frame
constexpr int kWideBlk = 4;        // Gram tiles per block side on the wide path (64 vars)
constexpr int kLdsRow = 66;        // padded LDS row (floats) of the per-wave E image

// contribution kinds for the assembly list
enum ContribKind : int {
  kEdgeBlock = 0,   // +H12(ro+r, co+c) of edge src
  kSchurBlock = 1,  // -S_f(6*ra+r, 6*rb+c)
  kEdgeRhs = 2,     // +v12(ro+r) of edge src
  kSchurRhs = 3,    // -S_f(6*ra+r, wcol)
};

// tile tasks of the dataflow Cholesky, 8 ints each: {type, i, j, k, a, b, c, 0}
//   kPotrf  i=j=k, a=klast, b=below, factor (k,k) after applying its last update
//           c=next+1, d=chained      (k,k,klast) itself (klast -1: none), store L_kk
//                                    and its diagonal-block inverses; below: also
//                                    solve tile (k+1,k); next: the ticket of
//                                    potrf(k+1), which this task then runs itself
//                                    (L(k+1,k) stays in LDS); chained: this ticket
//                                    is that placeholder (skipped when handed out)
//   kTrsm   i, j=k=k, a=seq, b=upd   tile (i,k) <- A_ik L_kk^-T (blocked forward
//                                    substitution); upd: then also the update
//                                    (i,k+1,k), the seq-th (and last) of (i,k+1)
//   kUpdate i, j, k, a=seq           tile (i,j) -= L_ik L_jk^T, its seq-th update
//   kBcol   i=j=k=c                  back solve of block c: x_c = L_cc^-T (y_c -
//                                    sum_{r>c} L_rc^T x_r), the x_r taken as they
//                                    are published, the parent's last
enum CholTaskType : int { kPotrf = 0, kTrsm = 1, kUpdate = 2, kBcol = 3 };
constexpr int kTaskInts = 8;

// The dataflow solve's sync area (zeroed before every launch): ticket, abort
// word, 2 spare ints, ver[nslots] | yver[nbc] | lkk[nbc], then (16-B aligned)
// the x hand-off granules {double x, int tag, int 0}, 64 per block column.
inline size_t chol_gran_off(int nslots, int nbc) { return ((size_t)(4 + nslots + 2 * nbc) * 4 + 15) & ~(size_t)15; }
inline size_t chol_sync_bytes(int nslots, int nbc) { return chol_gran_off(nslots, nbc) + (size_t)nbc * 64 * 16; }

struct Contrib {
  int kind, src, a0, a1;
};

// Tile-sparse structure of one factorisation: nbc pivot tile columns, nbr tile
// rows (the rhs is row n), slot[i*nbc+j] = storage slot of lower tile (i,j) or
// -1; fin[s] = final version of slot s (its update count + 1); ycnt[c] = final
// version of y_c (1: its forward-solved value; the back solve accumulates its
// updates inside the kBcol task).
struct CholStructure {
  int n = 0, nbc = 0, nbr = 0, nslots = 0, nslots_a = 0;
  std::vector<int> slot, fin, ycnt, tasks;
  int ntasks = 0;
  double cp = 0.0, work = 0.0;  // critical path and total cost of the task graph (task-cost units)
};

// pattern: lower tile (i,j) of the input system is nonzero; slots of these come
// first (the all-reduced region), fill tiles after.  Builds the fill closure
// and the task list in critical-path (bottom level) order.
void build_chol_structure(int n, const std::vector<char>& pattern, CholStructure& cs);

struct BaPlan {
  // problem
  int E = 0, N = 0, H = 0, W = 0, HW = 0;
  int t0 = 0, t1 = 0, P = 0, K = 0, n = 0;  // n = 6P
  int motion_only = 0, eta_rows = 0;
  int nsplit = 1;        // pixel splits per edge in ba_edge_hessian
  int group_per_wave = 1;
  int nchunk = 1;        // workgroups per frame in ba_frame_schur
  int nb_max = 1;        // largest tile count of a register-path frame
  int nb_all = 1;        // largest tile count of any frame
  // host arrays (all int32)
  std::vector<int> ii, jj;              // E
  std::vector<int> kx;                  // K
  std::vector<int> f_eptr, f_edges;     // K+1, E (edges grouped by source frame)
  std::vector<int> f_rptr, r_pose, r_edge;  // K+1, R, R
  std::vector<int> f_nb, f_goff;        // K, K (float offset of Gram partials)
  std::vector<int> wide_f, wide_eoff;   // frames on the wide path, float offset of their Ei image
  std::vector<int> wide_tasks;          // (wide index, IB, JB) per block pair
  long ei_floats = 0;
  std::vector<int> blk_a, blk_b, blk_cptr;  // nblk (permuted pose positions), nblk, nblk+1
  std::vector<int> rhs_cptr, rhs_pos;   // P+1, P (permuted position of each pose)
  std::vector<Contrib> contrib, rhs_contrib;
  long gram_floats = 0;
  // pose order: perm[a] = elimination position of pose a; outmap[v] = dx index of permuted var v
  std::vector<int> perm, outmap;
  int order_kind = 0;                   // 0 identity, 1 reverse Cuthill-McKee, 2 minimum degree, 3 nested dissection
  CholStructure cs;
  size_t sync_bytes = 0;                // ticket, abort, tile versions, y versions, x flags, L^-1 flags
  // device layout (byte offsets into the workspace)
  size_t off_ints = 0, off_hpart = 0, off_gram = 0, off_qw = 0, off_ei = 0, off_M = 0, off_x = 0,
         off_flag = 0, off_sync = 0, off_ybuf = 0, total = 0;
  // offsets (in ints) of each int array inside the int section
  size_t o_ii, o_jj, o_kx, o_feptr, o_fedges, o_frptr, o_rpose, o_redge, o_fnb, o_fgoff,
      o_blka, o_blkb, o_blkcptr, o_rhscptr, o_rhspos, o_contrib, o_rhscontrib, o_tasks,
      o_slot, o_fin, o_ycnt, o_outmap, o_widef, o_wideeoff, o_widetasks;
  std::vector<int> ints;  // packed int section, uploaded once
  bool uploaded = false;
  void* uploaded_to = nullptr;
};

}  // namespace droid
