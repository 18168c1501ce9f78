// Host-side structure analysis for one ba() call (the part of ba_cuda that
// depends only on ii, jj, t0, t1): droid_kernels.cu:1336-1345 (ts, kx, kk),
// :1241-1272 (Schur row graph) and the triplet lists of
// SparseBlock::update_lhs/rhs (:1131-1173), plus what SimplicialLLT's analyse
// step does for the reference (:1192-1213): a fill-reducing pose order and the
// symbolic factor, here at 64x64-tile granularity.  Unlike the reference, this
// runs once per edge set (cached by the caller), never inside the GN loop.
#include <algorithm>
#include <cstring>
#include <map>
#include <queue>
#include <unordered_map>
#include <utility>

#include "ba.hpp"
#include "common.hpp"

namespace droid {

static size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---------------------------------------------------------------------------
// Tile-level symbolic Cholesky.  Bitset per tile column: rows i >= j with
// nonzero (i, j).  Eliminating column k makes (i, j) nonzero for every pair of
// nonzero rows i >= j > k of column k.
// ---------------------------------------------------------------------------
struct TileBits {
  int nbc = 0, nbr = 0, nw = 0;
  std::vector<uint64_t> col;  // nbc x nw
  bool get(int i, int j) const { return (col[(size_t)j * nw + (i >> 6)] >> (i & 63)) & 1; }
  void set(int i, int j) { col[(size_t)j * nw + (i >> 6)] |= 1ull << (i & 63); }
};

static void init_bits(TileBits& tb, int n) {
  tb.nbc = (n + 63) / 64;
  tb.nbr = (n + 1 + 63) / 64;
  tb.nw = (tb.nbr + 63) / 64;
  tb.col.assign((size_t)tb.nbc * tb.nw, 0);
}

// diagonal tiles and the rhs row (row n: every column) are always present
static void close_bits(TileBits& tb) {
  for (int k = 0; k < tb.nbc; ++k) {
    tb.set(k, k);
    tb.set(tb.nbr - 1, k);
  }
  for (int k = 0; k < tb.nbc; ++k) {
    const uint64_t* ck = &tb.col[(size_t)k * tb.nw];
    for (int w = 0; w < tb.nw; ++w) {
      uint64_t bits = ck[w];
      while (bits) {
        const int i = 64 * w + __builtin_ctzll(bits);
        bits &= bits - 1;
        if (i <= k || i >= tb.nbc) continue;  // rows of column k that are also pivot columns j = i
        uint64_t* cj = &tb.col[(size_t)i * tb.nw];
        for (int w2 = i >> 6; w2 < tb.nw; ++w2) {
          uint64_t m = ck[w2];
          if (w2 == (i >> 6)) m &= ~0ull << (i & 63);
          cj[w2] |= m;
        }
      }
    }
  }
}

// number of tile updates the factorisation performs (its dominant work)
static long count_updates(const TileBits& tb) {
  long u = 0;
  for (int k = 0; k < tb.nbc; ++k) {
    long c = 0;
    for (int w = 0; w < tb.nw; ++w) c += __builtin_popcountll(tb.col[(size_t)k * tb.nw + w]);
    c -= 1;  // rows strictly below the diagonal
    u += c * (c + 1) / 2;
  }
  return u;
}

void build_chol_structure(int n, const std::vector<char>& pattern, CholStructure& cs) {
  TileBits tb;
  init_bits(tb, n);
  const int nbc = tb.nbc, nbr = tb.nbr;
  cs.n = n; cs.nbc = nbc; cs.nbr = nbr;
  cs.slot.assign((size_t)nbr * nbc, -1);
  cs.tasks.clear();
  cs.fin.clear(); cs.ycnt.assign(nbc, 1);
  cs.nslots = cs.nslots_a = 0;
  cs.ntasks = 0;
  if (n <= 0) return;
  std::vector<char> input((size_t)nbr * nbc, 0);
  for (int i = 0; i < nbr; ++i)
    for (int j = 0; j <= std::min(i, nbc - 1); ++j)
      if (pattern[(size_t)i * nbc + j] || i == j || i == nbr - 1) { input[(size_t)i * nbc + j] = 1; tb.set(i, j); }
  close_bits(tb);
  // slots: input tiles first (the region a sharded caller all-reduces), then fill
  for (int i = 0; i < nbr; ++i)
    for (int j = 0; j <= std::min(i, nbc - 1); ++j)
      if (input[(size_t)i * nbc + j]) cs.slot[(size_t)i * nbc + j] = cs.nslots++;
  cs.nslots_a = cs.nslots;
  for (int i = 0; i < nbr; ++i)
    for (int j = 0; j <= std::min(i, nbc - 1); ++j)
      if (tb.get(i, j) && cs.slot[(size_t)i * nbc + j] < 0) cs.slot[(size_t)i * nbc + j] = cs.nslots++;
  auto nz = [&](int i, int j) { return i >= 0 && j >= 0 && i < nbr && j < nbc && j <= i && cs.slot[(size_t)i * nbc + j] >= 0; };
  auto sl = [&](int i, int j) { return cs.slot[(size_t)i * nbc + j]; };
  // row bitsets (columns k of row i) for the update lists U(i,j) = {k < j : (i,k), (j,k) nonzero}
  const int cw = (nbc + 63) / 64;
  std::vector<uint64_t> rowb((size_t)nbr * cw, 0);
  for (int i = 0; i < nbr; ++i)
    for (int j = 0; j <= std::min(i, nbc - 1); ++j)
      if (nz(i, j)) rowb[(size_t)i * cw + (j >> 6)] |= 1ull << (j & 63);
  auto ulist = [&](int i, int j, std::vector<int>& out) {
    out.clear();
    for (int w = 0; w <= ((j - 1) >> 6) && j > 0; ++w) {
      uint64_t m = rowb[(size_t)i * cw + w] & rowb[(size_t)j * cw + w];
      if (w == (j >> 6)) m &= (1ull << (j & 63)) - 1;
      while (m) { out.push_back(64 * w + __builtin_ctzll(m)); m &= m - 1; }
    }
  };
  cs.fin.assign(cs.nslots, 1);
  std::vector<int> nupd(cs.nslots, 0), klast(nbc, -1);
  std::vector<int> U;
  for (int i = 0; i < nbr; ++i)
    for (int j = 0; j <= std::min(i, nbc - 1); ++j)
      if (nz(i, j)) {
        ulist(i, j, U);
        nupd[sl(i, j)] = (int)U.size();
        cs.fin[sl(i, j)] = (int)U.size() + 1;
        if (i == j && !U.empty()) klast[i] = U.back();
      }
  // back-solve rows of each x_c (the nonzero tiles below its diagonal), descending
  std::vector<std::vector<int>> yrows(nbc);
  for (int c = 0; c < nbc; ++c)
    for (int r = nbc - 1; r > c; --r)
      if (nz(r, c)) yrows[c].push_back(r);
  cs.ycnt.assign(nbc, 1);   // y_c: only its forward-solved value is published (version 1)

  // ---- task graph ----
  struct Node { int rec[kTaskInts]; double cost; std::vector<int> succ; int npred; double bl; };
  std::vector<Node> t;
  std::unordered_map<uint64_t, int> id;
  auto key = [](int type, int i, int j, int k) {
    return (uint64_t)type | ((uint64_t)(uint32_t)i << 4) | ((uint64_t)(uint32_t)j << 24) | ((uint64_t)(uint32_t)k << 44);
  };
  auto add = [&](int type, int i, int j, int k, int a, int b, int c, double cost) {
    id[key(type, i, j, k)] = (int)t.size();
    Node nd{{type, i, j, k, a, b, c, 0}, cost, {}, 0, 0.0};
    t.push_back(std::move(nd));
  };
  // potrf(k) also solves tile (k+1,k) when it exists
  std::vector<char> below(nbc, 0);
  auto fused = [&](int i, int k) { return i == k + 1 && below[k]; };
  for (int k = 0; k < nbc; ++k)
    below[k] = (k + 1 < nbr && nz(k + 1, k)) ? 1 : 0;
  // trsm(i,k) also applies the update (i,k+1,k) - always the last of tile
  // (i,k+1) - when tile (k+1,k) exists: fusedu(i,k)
  auto fusedu = [&](int i, int k) { return k + 1 < nbc && i > k + 1 && below[k] && nz(i, k + 1); };
  for (int k = 0; k < nbc; ++k) {
    add(kPotrf, k, k, k, klast[k], below[k], 0, 10.0);
    for (int i = k + 1; i < nbr; ++i)
      if (nz(i, k) && !fused(i, k)) {
        int seq = 0;
        if (fusedu(i, k)) { ulist(i, k + 1, U); seq = (int)U.size() - 1; }
        add(kTrsm, i, k, k, seq, fusedu(i, k) ? 1 : 0, 0, 2.0);
      }
  }
  for (int i = 0; i < nbr; ++i)
    for (int j = 0; j <= std::min(i, nbc - 1); ++j)
      if (nz(i, j)) {
        ulist(i, j, U);
        for (int s = 0; s < (int)U.size(); ++s)
          if (!(i == j && U[s] == klast[i]) && !(U[s] == j - 1 && fusedu(i, j - 1))) add(kUpdate, i, j, U[s], s, 0, 0, 2.0);
      }
  for (int c = 0; c < nbc; ++c) add(kBcol, c, c, c, 0, 0, 0, 2.0);
  auto get = [&](int type, int i, int j, int k) { return id.at(key(type, i, j, k)); };
  auto fin_task = [&](int i, int k) {  // the task that makes tile (i,k) final
    if (i == k || fused(i, k)) return get(kPotrf, k, k, k);
    return get(kTrsm, i, k, k);
  };
  auto upd_task = [&](int i, int j, int s) {  // the task that publishes version s+1 of (i,j)
    ulist(i, j, U);
    if (U[s] == j - 1 && fusedu(i, j - 1)) return get(kTrsm, i, j - 1, j - 1);
    return get(kUpdate, i, j, U[s]);
  };
  auto edge = [&](int a, int b) {
    for (int x : t[a].succ)
      if (x == b) return;
    t[a].succ.push_back(b);
    t[b].npred++;
  };
  for (int v = 0; v < (int)t.size(); ++v) {
    const int type = t[v].rec[0], i = t[v].rec[1], j = t[v].rec[2], k = t[v].rec[3], a = t[v].rec[4];
    switch (type) {
      case kPotrf: {
        const int nu = nupd[sl(k, k)];
        if (nu >= 2) edge(upd_task(k, k, nu - 2), v);
        if (a >= 0) edge(fin_task(k, a), v);
        if (t[v].rec[5] && nupd[sl(k + 1, k)] >= 1)   // the fused tile's last update (awaited inside the task)
          edge(upd_task(k + 1, k, nupd[sl(k + 1, k)] - 1), v);
        break;
      }
      case kTrsm:
        edge(get(kPotrf, k, k, k), v);
        if (nupd[sl(i, k)] >= 1) edge(upd_task(i, k, nupd[sl(i, k)] - 1), v);
        if (t[v].rec[5] && a >= 1) edge(upd_task(i, k + 1, a - 1), v);   // the fused update's predecessor
        break;
      case kUpdate:
        if (a >= 1) edge(upd_task(i, j, a - 1), v);
        edge(fin_task(i, k), v);
        edge(fin_task(j, k), v);
        break;
      default:  // kBcol (c = i): L_cc^-1, y_c's forward value, the tiles below and their x_r
        edge(get(kPotrf, i, i, i), v);
        edge(fin_task(nbr - 1, i), v);
        for (int r : yrows[i]) {
          edge(fin_task(r, i), v);
          edge(get(kBcol, r, r, r), v);
        }
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
  cs.cp = cs.work = 0.0;
  for (int q = (int)order.size() - 1; q >= 0; --q) {
    Node& nd = t[order[q]];
    double m = 0.0;
    for (int s2 : nd.succ) m = std::max(m, 1.0 + t[s2].bl);
    nd.bl = nd.cost + m;
    cs.cp = std::max(cs.cp, nd.bl);
    cs.work += nd.cost;
  }
  // list scheduling by bottom level: tickets are a topological order, so a
  // task never waits on one that has not been handed out
  auto cmp = [&](int a, int b) { return t[a].bl != t[b].bl ? t[a].bl < t[b].bl : a > b; };
  std::priority_queue<int, std::vector<int>, decltype(cmp)> ready(cmp);
  for (size_t v = 0; v < t.size(); ++v) {
    indeg[v] = t[v].npred;
    if (!indeg[v]) ready.push((int)v);
  }
  std::vector<int> ticket(t.size(), -1);
  while (!ready.empty()) {
    const int v = ready.top();
    ready.pop();
    ticket[v] = (int)cs.tasks.size() / kTaskInts;
    cs.tasks.insert(cs.tasks.end(), t[v].rec, t[v].rec + kTaskInts);
    for (int s2 : t[v].succ)
      if (--indeg[s2] == 0) ready.push(s2);
  }
  cs.ntasks = (int)cs.tasks.size() / kTaskInts;
  // Chains of pivots: potrf(k) runs potrf(k+1) itself when tile (k+1,k) is
  // solved in potrf(k) and is the last update of (k+1,k+1) - L(k+1,k) stays in
  // LDS.  potrf(k+1)'s ticket stays in the list as a placeholder, so the list
  // is still a topological order (a task never waits on one not yet handed out).
  for (int k = 0; k + 1 < nbc; ++k)
    if (below[k] && klast[k + 1] == k) {
      const int a = ticket[get(kPotrf, k, k, k)], b = ticket[get(kPotrf, k + 1, k + 1, k + 1)];
      cs.tasks[(size_t)a * kTaskInts + 6] = b + 1;
      cs.tasks[(size_t)b * kTaskInts + 7] = 1;
    }
}

// ---------------------------------------------------------------------------
// Pose orderings for the reduced system (adjacency of poses sharing a block).
// ---------------------------------------------------------------------------
static std::vector<int> order_rcm(int P, const std::vector<std::vector<int>>& adj) {
  std::vector<int> deg(P), out;
  for (int a = 0; a < P; ++a) deg[a] = (int)adj[a].size();
  std::vector<char> done(P, 0);
  std::vector<int> lvl(P);
  auto bfs = [&](int s, std::vector<int>& seq, bool mark) {
    std::vector<char> seen(P, 0);
    seq.clear();
    seq.push_back(s); seen[s] = 1; lvl[s] = 0;
    for (size_t q = 0; q < seq.size(); ++q) {
      std::vector<int> nb;
      for (int b : adj[seq[q]]) if (!seen[b] && !done[b]) nb.push_back(b);
      std::sort(nb.begin(), nb.end(), [&](int x, int y) { return deg[x] != deg[y] ? deg[x] < deg[y] : x < y; });
      for (int b : nb) { seen[b] = 1; lvl[b] = lvl[seq[q]] + 1; seq.push_back(b); }
    }
    if (mark) for (int v : seq) done[v] = 1;
  };
  std::vector<int> seq;
  for (int s0 = 0; s0 < P; ++s0) {
    if (done[s0]) continue;
    // pseudo-peripheral start: repeat BFS from the farthest, lowest-degree node
    int s = s0, ecc = -1;
    for (int it = 0; it < 4; ++it) {
      bfs(s, seq, false);
      const int e = lvl[seq.back()];
      if (e <= ecc) break;
      ecc = e;
      int best = seq.back();
      for (int v : seq) if (lvl[v] == e && deg[v] < deg[best]) best = v;
      s = best;
    }
    bfs(s, seq, true);
    out.insert(out.end(), seq.begin(), seq.end());
  }
  std::reverse(out.begin(), out.end());
  std::vector<int> perm(P);
  for (int q = 0; q < P; ++q) perm[out[q]] = q;
  return perm;
}

static std::vector<int> order_mindeg(int P, const std::vector<std::vector<int>>& adj) {
  const int nw = (P + 63) / 64;
  std::vector<uint64_t> g((size_t)P * nw, 0);
  for (int a = 0; a < P; ++a)
    for (int b : adj[a]) g[(size_t)a * nw + (b >> 6)] |= 1ull << (b & 63);
  std::vector<int> deg(P), perm(P, -1);
  std::vector<char> alive(P, 1);
  for (int a = 0; a < P; ++a) deg[a] = (int)adj[a].size();
  std::vector<int> nb;
  for (int q = 0; q < P; ++q) {
    int v = -1;
    for (int a = 0; a < P; ++a)
      if (alive[a] && (v < 0 || deg[a] < deg[v])) v = a;
    perm[v] = q;
    alive[v] = 0;
    nb.clear();
    for (int w = 0; w < nw; ++w) {
      uint64_t m = g[(size_t)v * nw + w];
      while (m) { const int b = 64 * w + __builtin_ctzll(m); m &= m - 1; if (alive[b]) nb.push_back(b); }
    }
    for (int b : nb) {
      uint64_t* gb = &g[(size_t)b * nw];
      const uint64_t* gv = &g[(size_t)v * nw];
      int d = 0;
      for (int w = 0; w < nw; ++w) gb[w] |= gv[w];
      gb[b >> 6] &= ~(1ull << (b & 63));
      gb[v >> 6] &= ~(1ull << (v & 63));
      for (int w = 0; w < nw; ++w) {
        uint64_t m = gb[w];
        while (m) { const int c = 64 * w + __builtin_ctzll(m); m &= m - 1; d += alive[c]; }
      }
      deg[b] = d;
    }
  }
  return perm;
}

// Nested dissection on 64-variable tile boundaries: a block of poses is ordered
// [ND(A), ND(B), S], A = the first m poses of a breadth-first sweep from a
// pseudo-peripheral pose (m near half, chosen so that B starts on a tile
// boundary: 6 (base + m) = 0 mod 64), S = the poses outside A adjacent to it
// (a vertex separator), B = the rest.  A and B then share no tile column, so
// their factorisations are independent subtrees and the Cholesky's critical
// path is the tree height instead of the whole band (a lapping trajectory's
// revisit edges make the reduced system a banded cylinder whose band RCM cannot
// narrow).
static void nd_block(std::vector<int> nodes, int base, const std::vector<std::vector<int>>& adj,
                     std::vector<int>& region, int& rid, std::vector<int>& out) {
  constexpr int kLeaf = 32;  // poses per tile-aligned leaf (= 3 tiles)
  const int sz = (int)nodes.size();
  if (sz <= kLeaf) {
    std::sort(nodes.begin(), nodes.end());
    out.insert(out.end(), nodes.begin(), nodes.end());
    return;
  }
  const int me = ++rid;
  for (int v : nodes) region[v] = me;
  std::vector<int> lvl(adj.size(), -1);
  auto bfs = [&](int s, std::vector<int>& seq) {
    seq.clear();
    for (int v : nodes) lvl[v] = -1;
    seq.push_back(s);
    lvl[s] = 0;
    for (size_t q = 0; q < seq.size(); ++q)
      for (int b : adj[seq[q]])
        if (region[b] == me && lvl[b] < 0) { lvl[b] = lvl[seq[q]] + 1; seq.push_back(b); }
  };
  std::vector<int> seq;
  bfs(*std::min_element(nodes.begin(), nodes.end()), seq);
  if ((int)seq.size() < sz) {  // disconnected: the components one after another
    std::vector<int> rest;
    for (int v : nodes) if (lvl[v] < 0) rest.push_back(v);
    std::vector<int> comp = seq;
    nd_block(comp, base, adj, region, rid, out);
    for (int v : rest) region[v] = me;  // (the call above re-tagged its own nodes)
    nd_block(rest, base + (int)comp.size(), adj, region, rid, out);
    return;
  }
  for (int it = 0; it < 3; ++it) {  // pseudo-peripheral start
    const int far = seq.back();
    std::vector<int> s2;
    bfs(far, s2);
    if (lvl[s2.back()] <= lvl[seq.back()] && it > 0) break;
    seq.swap(s2);
  }
  // m: B's first pose on a tile boundary, as close to half as possible
  int m = -1;
  for (int c = ((base + sz / 2) / 32) * 32 - base, d = 0; d <= sz; d += 32) {
    for (int cand : {c + d, c - d + 32, c - d})
      if (cand >= kLeaf / 2 && cand <= sz - kLeaf / 2 && (m < 0 || std::abs(cand - sz / 2) < std::abs(m - sz / 2)))
        m = cand;
    if (m >= 0) break;
  }
  if (m < 0) {
    std::sort(nodes.begin(), nodes.end());
    out.insert(out.end(), nodes.begin(), nodes.end());
    return;
  }
  std::vector<char> inA(adj.size(), 0);
  for (int q = 0; q < m; ++q) inA[seq[q]] = 1;
  std::vector<int> A(seq.begin(), seq.begin() + m), B, S;
  for (int q = m; q < sz; ++q) {
    const int v = seq[q];
    bool sep = false;
    for (int b : adj[v]) if (region[b] == me && inA[b]) { sep = true; break; }
    (sep ? S : B).push_back(v);
  }
  if (B.empty()) {
    std::sort(nodes.begin(), nodes.end());
    out.insert(out.end(), nodes.begin(), nodes.end());
    return;
  }
  nd_block(A, base, adj, region, rid, out);
  nd_block(B, base + m, adj, region, rid, out);
  std::sort(S.begin(), S.end());
  out.insert(out.end(), S.begin(), S.end());
}

static std::vector<int> order_nd(int P, const std::vector<std::vector<int>>& adj) {
  std::vector<int> nodes(P), out, region(P, 0);
  for (int a = 0; a < P; ++a) nodes[a] = a;
  int rid = 0;
  nd_block(nodes, 0, adj, region, rid, out);
  std::vector<int> perm(P);
  for (int q = 0; q < P; ++q) perm[out[q]] = q;
  return perm;
}

static void tile_pattern(int n, int P, const std::vector<int>& perm, const std::vector<std::pair<int, int>>& pairs,
                         std::vector<char>& pat) {
  const int nbc = (n + 63) / 64, nbr = (n + 1 + 63) / 64;
  pat.assign((size_t)nbr * nbc, 0);
  auto mark = [&](int pa, int pb) {  // 6x6 block at permuted pose positions pa >= pb
    for (int ti = (6 * pa) >> 6; ti <= (6 * pa + 5) >> 6; ++ti)
      for (int tj = (6 * pb) >> 6; tj <= (6 * pb + 5) >> 6; ++tj)
        if (tj <= ti) pat[(size_t)ti * nbc + tj] = 1;
  };
  for (int a = 0; a < P; ++a) mark(perm[a], perm[a]);
  for (auto& pr : pairs) {
    const int pa = perm[pr.first], pb = perm[pr.second];
    mark(std::max(pa, pb), std::min(pa, pb));
  }
}

// the reduced system's pose-pair pattern: edge blocks (i,j) and Schur blocks of
// every pair of optimised rows sharing a depth frame (the global graph, so every
// rank of a sharded BA derives the same structure)
static void pose_pairs(const std::vector<int>& gi, const std::vector<int>& gj, int t0, int t1,
                       std::vector<std::pair<int, int>>& pairs, int motion_only) {
  const int P = t1 - t0;
  std::vector<std::vector<int>> rows;  // optimised poses per depth frame
  std::map<int, int> fidx;
  pairs.clear();
  for (size_t e = 0; e < gi.size(); ++e) {
    const int a = gi[e] - t0, b = gj[e] - t0;
    if (a >= 0 && a < P && b >= 0 && b < P && a != b) pairs.push_back({std::max(a, b), std::min(a, b)});
  }
  if (!motion_only) {
    for (size_t e = 0; e < gi.size(); ++e) {
      auto it = fidx.find(gi[e]);
      int f;
      if (it == fidx.end()) {
        f = (int)rows.size();
        fidx[gi[e]] = f;
        rows.push_back({});
        if (gi[e] >= t0 && gi[e] < t1) rows[f].push_back(gi[e] - t0);
      } else {
        f = it->second;
      }
      if (gj[e] >= t0 && gj[e] < t1) rows[f].push_back(gj[e] - t0);
    }
    for (auto& r : rows) {
      std::sort(r.begin(), r.end());
      r.erase(std::unique(r.begin(), r.end()), r.end());
      for (size_t x = 0; x < r.size(); ++x)
        for (size_t y = 0; y < x; ++y) pairs.push_back({r[x], r[y]});
    }
  }
  std::sort(pairs.begin(), pairs.end());
  pairs.erase(std::unique(pairs.begin(), pairs.end()), pairs.end());
}

// tile updates of the factorisation under a pose order (its dominant work)
static long order_updates(int n, int P, const std::vector<int>& perm, const std::vector<std::pair<int, int>>& pairs) {
  std::vector<char> pat;
  tile_pattern(n, P, perm, pairs, pat);
  TileBits tb;
  init_bits(tb, n);
  for (int i = 0; i < tb.nbr; ++i)
    for (int j = 0; j <= std::min(i, tb.nbc - 1); ++j)
      if (pat[(size_t)i * tb.nbc + j]) tb.set(i, j);
  close_bits(tb);
  return count_updates(tb);
}

// The pose order: the candidate whose task graph the dataflow Cholesky (one
// persistent workgroup per CU) is expected to finish first, i.e. the smaller of
// max(critical path, work / workers) in task-cost units; the identity is kept
// unless a candidate beats it by more than 5 %.
static double chol_makespan(int n, int P, const std::vector<int>& perm, const std::vector<std::pair<int, int>>& pairs) {
  constexpr double kWorkers = 256.0;
  std::vector<char> pat;
  tile_pattern(n, P, perm, pairs, pat);
  CholStructure cs;
  build_chol_structure(n, pat, cs);
  return std::max(cs.cp, cs.work / kWorkers);
}

// forced pose order for new plans (droid_ba_set_order): -1 = chosen by the
// plan (default), 0 identity, 1 rcm, 2 mindeg, 3 nd (A/B runs and tests)
static int g_force_order = -1;

static void choose_order(BaPlan& p, const std::vector<std::pair<int, int>>& pairs) {
  const int P = p.P, n = p.n;
  std::vector<int> ident(P);
  for (int a = 0; a < P; ++a) ident[a] = a;
  p.perm = ident;
  p.order_kind = 0;
  const int force = g_force_order;
  if (P <= 32 && force < 0) return;                  // a handful of tiles: nothing to gain
  std::vector<std::vector<int>> adj(P);
  for (auto& pr : pairs) { adj[pr.first].push_back(pr.second); adj[pr.second].push_back(pr.first); }
  auto make = [&](int kind) {
    return kind == 1 ? order_rcm(P, adj) : kind == 2 ? order_mindeg(P, adj) : order_nd(P, adj);
  };
  if (force >= 0) {
    if (force) { p.perm = make(force); p.order_kind = force; }
    return;
  }
  // the task graph (the critical path) is built only for orders whose tile
  // update count is within 4x of the fewest: a fill-heavy order's graph is
  // large (~1M tasks for the identity at C5) and never the fastest
  const bool verbose = ab_knob("DROID_BA_PLAN_VERBOSE", 0) != 0;
  std::vector<std::vector<int>> perms(4);
  std::vector<long> upd(4);
  perms[0] = ident;
  for (int kind = 0; kind <= 3; ++kind) {
    if (kind) perms[kind] = make(kind);
    upd[kind] = order_updates(n, P, perms[kind], pairs);
  }
  const long umin = *std::min_element(upd.begin(), upd.end());
  double keep = -1.0, best = -1.0;
  for (int kind = 0; kind <= 3; ++kind) {
    if (upd[kind] > 4 * umin + 64) continue;
    const double c = chol_makespan(n, P, perms[kind], pairs);
    if (verbose) fprintf(stderr, "ba plan P=%d order %d: %ld tile updates, makespan %.0f\n", P, kind, upd[kind], c);
    if (kind == 0) { keep = best = c; continue; }
    if (best < 0 || (c < best && (keep < 0 || c * 20 < keep * 19))) {
      best = c;
      p.perm = perms[kind];
      p.order_kind = kind;
    }
  }
}

static int build_plan(BaPlan& p, const int64_t* ii, const int64_t* jj, int E, const int64_t* gii,
                      const int64_t* gjj, int gE, int N, int H, int W, int t0, int t1, int eta_rows,
                      int motion_only, int own_lo, int own_hi) {
  if (E < 0 || gE < 0 || N <= 0 || H <= 0 || W <= 0) return fail(kInvalidArgument, "ba: bad sizes");
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
  std::vector<int> gi(gE), gj(gE);
  for (int e = 0; e < gE; ++e) {
    if (gii[e] < 0 || gii[e] >= N || gjj[e] < 0 || gjj[e] >= N)
      return fail(kInvalidArgument, "ba: global edge index out of range");
    gi[e] = (int)gii[e];
    gj[e] = (int)gjj[e];
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
  // pixel splits per edge: enough (edge, split) workgroups to cover the CUs
  // (~512), but few enough that each sums >= 256 pixels before its 90-partial
  // reduction and the assembly does not sum many partials per element
  // pixel splits per edge: ~192 (edge, split) workgroups for small graphs.  A/B
  // on one MI355X (DROID_BA_NSPLIT, profiles/r02/ba_nsplit_r02dj.txt): C2 (96
  // edges) BA(itrs=2) 0.209 ms at 2 splits vs 0.242 at 6 (the old 512-workgroup
  // target) and 0.281 at 12; C3 is fastest unsplit (2.41 vs 2.52 ms at 2)
  p.nsplit = std::max(1, std::min(std::max(1, HW / 256), (192 + std::max(E, 1) - 1) / std::max(E, 1)));
  if (const int f = ab_knob("DROID_BA_NSPLIT", 0)) p.nsplit = std::max(1, std::min(std::max(1, HW / 64), f));
  const int rounds = ceil_div(HW, 256);
  p.group_per_wave = std::max(1, std::min(rounds, (int)((long)p.K * rounds / 1024)));
  p.nchunk = ceil_div(rounds, p.group_per_wave);

  // Schur rows per frame: [Ei row if the frame's pose is optimised] + one Eij row per edge.
  // Frames whose Gram fits the register tile (<= kNbMax tiles a side) take the
  // one-kernel path; the others the wide (prep + blocked Gram) path.
  p.f_rptr.assign(p.K + 1, 0);
  p.r_pose.clear(); p.r_edge.clear();
  p.f_nb.assign(p.K, 0); p.f_goff.assign(p.K, 0);
  p.wide_f.clear(); p.wide_eoff.clear(); p.wide_tasks.clear();
  p.nb_max = 1; p.nb_all = 1;
  p.gram_floats = 0; p.ei_floats = 0;
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
    p.f_nb[f] = nb;
    p.nb_all = std::max(p.nb_all, nb);
    if (nb > kNbMax) {
      const int w = (int)p.wide_f.size();
      p.wide_f.push_back(f);
      p.wide_eoff.push_back((int)p.ei_floats);
      p.ei_floats += 6L * HW;
      const int nblk = ceil_div(nb, kWideBlk);
      for (int a = 0; a < nblk; ++a)
        for (int b = a; b < nblk; ++b) { p.wide_tasks.push_back(w); p.wide_tasks.push_back(a); p.wide_tasks.push_back(b); }
    } else {
      p.nb_max = std::max(p.nb_max, nb);
    }
    p.f_goff[f] = (int)p.gram_floats;
    p.gram_floats += (long)p.nchunk * (nb * (nb + 1) / 2) * 256;
  }
  if (p.gram_floats > 0x7fffffffL || p.ei_floats > 0x7fffffffL)
    return fail(kUnsupported, "ba: Schur workspace exceeds 2^31 floats");
  if (motion_only) { p.gram_floats = 0; p.ei_floats = 0; p.wide_f.clear(); p.wide_eoff.clear(); p.wide_tasks.clear(); }

  // pose order + tile structure of the factor (from the global graph)
  const int P = p.P;
  std::vector<std::pair<int, int>> pairs;
  pose_pairs(gi, gj, t0, t1, pairs, motion_only);
  choose_order(p, pairs);
  {
    std::vector<char> pat;
    tile_pattern(p.n, P, p.perm, pairs, pat);
    build_chol_structure(p.n, pat, p.cs);
  }
  std::vector<int> iperm(P);
  for (int a = 0; a < P; ++a) iperm[p.perm[a]] = a;
  p.outmap.assign(p.n, 0);
  for (int v = 0; v < p.n; ++v) p.outmap[v] = 6 * iperm[v / 6] + v % 6;
  p.rhs_pos = p.perm;

  // Block contribution lists for the lower triangle of the reduced system
  // (original pose indices r >= c; the kernel maps them to permuted positions).
  std::map<std::pair<int, int>, std::vector<Contrib>> blocks;
  std::vector<std::vector<Contrib>> rhs(P);
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
  // Every block the assembly writes must land in an input tile of the factor's
  // structure (the region a sharded caller all-reduces).  The structure comes
  // from the global edge list, so a rank whose local edges are not part of it
  // would otherwise write through slot -1 or into a fill tile.
  {
    const int nbc = p.cs.nbc;
    auto covered = [&](int v, int u) {
      const int s = p.cs.slot[(size_t)(v >> 6) * nbc + (u >> 6)];
      return s >= 0 && s < p.cs.nslots_a;
    };
    for (auto& kv : blocks) {
      const int pa = p.perm[kv.first.first], pb = p.perm[kv.first.second];
      for (int r = 0; r < 6; ++r)
        for (int c = 0; c < 6; ++c) {
          const int v = 6 * pa + r, u = 6 * pb + c;
          if (!(v >= u ? covered(v, u) : (pa == pb || covered(u, v))))
            return fail(kInvalidArgument, "ba: local edges not covered by the global edge list");
        }
    }
    for (int a = 0; a < P; ++a)
      if (!rhs[a].empty())
        for (int c = 0; c < 6; ++c)
          if (!covered(p.n, 6 * p.perm[a] + c))
            return fail(kInvalidArgument, "ba: local edges not covered by the global edge list");
  }
  p.blk_a.clear(); p.blk_b.clear(); p.blk_cptr.assign(1, 0); p.contrib.clear();
  for (auto& kv : blocks) {
    p.blk_a.push_back(p.perm[kv.first.first]);
    p.blk_b.push_back(p.perm[kv.first.second]);
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
  p.o_rhscptr = put(p.rhs_cptr); p.o_rhspos = put(p.rhs_pos);
  p.o_contrib = putc(p.contrib); p.o_rhscontrib = putc(p.rhs_contrib);
  p.o_tasks = put(p.cs.tasks);
  p.o_slot = put(p.cs.slot); p.o_fin = put(p.cs.fin); p.o_ycnt = put(p.cs.ycnt);
  p.o_outmap = put(p.outmap);
  p.o_widef = put(p.wide_f); p.o_wideeoff = put(p.wide_eoff); p.o_widetasks = put(p.wide_tasks);
  if (p.ints.empty()) p.ints.push_back(0);
  const int nbc = p.cs.nbc;
  p.sync_bytes = chol_sync_bytes(p.cs.nslots, nbc);
  if ((size_t)std::max(p.cs.nslots, 1) * kTile * 8 >= 0x80000000ull)
    return fail(kUnsupported, "ba: factor tiles exceed the 2 GB buffer-resource range");

  // workspace layout
  size_t off = 0;
  p.off_ints = off; off = align_up(off + p.ints.size() * 4, 256);
  p.off_hpart = off; off = align_up(off + (size_t)std::max(E, 1) * p.nsplit * kHessStride * 4, 256);
  p.off_gram = off; off = align_up(off + (size_t)std::max(p.gram_floats, 1L) * 4, 256);
  p.off_qw = off; off = align_up(off + (size_t)2 * p.K * HW * 4 + 4, 256);
  p.off_ei = off; off = align_up(off + (size_t)std::max(p.ei_floats, 1L) * 4, 256);
  p.off_M = off; off = align_up(off + (size_t)std::max(p.cs.nslots, 1) * kTile * 8, 256);
  p.off_x = off; off = align_up(off + (size_t)(p.n + 1) * 8, 256);
  p.off_flag = off; off = align_up(off + 64, 256);
  p.off_sync = off; off = align_up(off + p.sync_bytes, 256);
  p.off_ybuf = off; off = align_up(off + (size_t)std::max(nbc, 1) * 64 * 8, 256);
  p.total = off;
  return kOk;
}

}  // namespace droid

using namespace droid;

extern "C" {

// Sharded BA: ii/jj are this rank's edges; gii/gjj the global edge list, from
// which the pose order and the factor's tile structure are derived (identical
// on every rank, so the reduced systems line up for the all-reduce).
int droid_ba_plan_create_sharded(const int64_t* ii, const int64_t* jj, int num_edges, const int64_t* gii,
                                 const int64_t* gjj, int num_global_edges, int num_frames, int ht, int wd, int t0,
                                 int t1, int eta_rows, int motion_only, int own_lo, int own_hi, void** plan_out) {
  if (!plan_out) return fail(kInvalidArgument, "ba_plan_create: null output");
  *plan_out = nullptr;
  auto* p = new BaPlan();
  int st = build_plan(*p, ii, jj, num_edges, gii, gjj, num_global_edges, num_frames, ht, wd, t0, t1, eta_rows,
                      motion_only, own_lo, own_hi);
  if (st != kOk) { delete p; return st; }
  *plan_out = p;
  return kOk;
}

int droid_ba_plan_create(const int64_t* ii, const int64_t* jj, int num_edges, int num_frames,
                         int ht, int wd, int t0, int t1, int eta_rows, int motion_only,
                         int own_lo, int own_hi, void** plan_out) {
  return droid_ba_plan_create_sharded(ii, jj, num_edges, ii, jj, num_edges, num_frames, ht, wd, t0, t1, eta_rows,
                                      motion_only, own_lo, own_hi, plan_out);
}

// Dense SPD solve of an n x n system on the dataflow Cholesky alone (no BA):
// every lower tile present, identity order.  droid_chol_set_system loads A, b.
int droid_chol_plan_create(int n, void** plan_out) {
  if (!plan_out || n < 0) return fail(kInvalidArgument, "chol_plan_create: bad arguments");
  auto* p = new BaPlan();
  p->n = n;
  p->P = 0;
  p->motion_only = 1;
  const int nbc = (n + 63) / 64, nbr = (n + 1 + 63) / 64;
  std::vector<char> pat((size_t)nbr * nbc, 1);
  build_chol_structure(n, pat, p->cs);
  p->outmap.resize(n);
  for (int v = 0; v < n; ++v) p->outmap[v] = v;
  p->ints.clear();
  auto put = [&](const std::vector<int>& v) {
    size_t o = p->ints.size();
    p->ints.insert(p->ints.end(), v.begin(), v.end());
    while (p->ints.size() % 4) p->ints.push_back(0);
    return o;
  };
  p->o_tasks = put(p->cs.tasks);
  p->o_slot = put(p->cs.slot); p->o_fin = put(p->cs.fin); p->o_ycnt = put(p->cs.ycnt);
  p->o_outmap = put(p->outmap);
  if (p->ints.empty()) p->ints.push_back(0);
  p->sync_bytes = chol_sync_bytes(p->cs.nslots, nbc);
  size_t off = 0;
  p->off_ints = off; off = align_up(off + p->ints.size() * 4, 256);
  p->off_M = off; off = align_up(off + (size_t)std::max(p->cs.nslots, 1) * kTile * 8, 256);
  p->off_x = off; off = align_up(off + (size_t)(n + 1) * 8, 256);
  p->off_flag = off; off = align_up(off + 64, 256);
  p->off_sync = off; off = align_up(off + p->sync_bytes, 256);
  p->off_ybuf = off; off = align_up(off + (size_t)std::max(nbc, 1) * 64 * 8, 256);
  p->total = off;
  *plan_out = p;
  return kOk;
}

// ntasks, the flag word's byte offset in the workspace, tile slots (all / input region)
int droid_chol_plan_info(const void* plan, int* ntasks, int* flag_offset, int* nslots, int* nslots_input) {
  auto* p = static_cast<const BaPlan*>(plan);
  if (!p) return fail(kInvalidArgument, "chol_plan_info: null plan");
  if (ntasks) *ntasks = p->cs.ntasks;
  if (flag_offset) *flag_offset = (int)p->off_flag;
  if (nslots) *nslots = p->cs.nslots;
  if (nslots_input) *nslots_input = p->cs.nslots_a;
  return kOk;
}

// the plan's Cholesky task list in ticket order (kTaskInts ints per task)
int droid_chol_plan_tasks(const void* plan, int* out) {
  auto* p = static_cast<const BaPlan*>(plan);
  if (!p || !out) return fail(kInvalidArgument, "chol_plan_tasks: null argument");
  std::copy(p->cs.tasks.begin(), p->cs.tasks.end(), out);
  return kOk;
}

// slot map (nbr*nbc ints, -1 = structural zero), final tile versions (nslots),
// final y versions (nbc), and the permuted-var -> dx index map (n)
int droid_chol_plan_structure(const void* plan, int* slot, int* fin, int* ycnt, int* outmap) {
  auto* p = static_cast<const BaPlan*>(plan);
  if (!p) return fail(kInvalidArgument, "chol_plan_structure: null plan");
  if (slot) std::copy(p->cs.slot.begin(), p->cs.slot.end(), slot);
  if (fin) std::copy(p->cs.fin.begin(), p->cs.fin.end(), fin);
  if (ycnt) std::copy(p->cs.ycnt.begin(), p->cs.ycnt.end(), ycnt);
  if (outmap) std::copy(p->outmap.begin(), p->outmap.end(), outmap);
  return kOk;
}

void droid_ba_plan_destroy(void* plan) { delete static_cast<BaPlan*>(plan); }

// Pose order of the plans created from now on: -1 = chosen per plan by the
// expected dataflow makespan (default), 0 identity, 1 reverse Cuthill-McKee,
// 2 minimum degree, 3 nested dissection.  Returns the previous setting, or -2
// for a mode outside -1..3.  Process-wide (tests and A/B runs).
int droid_ba_set_order(int kind) {
  if (kind < -1 || kind > 3) return -2;
  const int prev = g_force_order;
  g_force_order = kind;
  return prev;
}

size_t droid_ba_plan_workspace_bytes(const void* plan) {
  return plan ? static_cast<const BaPlan*>(plan)->total : 0;
}

int droid_ba_plan_info(const void* plan, int* K, int* P, int* nblocks, int* nb_max) {
  auto* p = static_cast<const BaPlan*>(plan);
  if (!p) return fail(kInvalidArgument, "ba_plan_info: null plan");
  if (K) *K = p->K;
  if (P) *P = p->P;
  if (nblocks) *nblocks = (int)p->blk_a.size();
  if (nb_max) *nb_max = p->nb_all;
  return kOk;
}

// order kind (0 identity, 1 RCM, 2 min degree), the pose order (P ints),
// number of wide-path frames and tile tasks
int droid_ba_plan_order(const void* plan, int* kind, int* perm, int* num_wide, int* ntasks) {
  auto* p = static_cast<const BaPlan*>(plan);
  if (!p) return fail(kInvalidArgument, "ba_plan_order: null plan");
  if (kind) *kind = p->order_kind;
  if (perm) std::copy(p->perm.begin(), p->perm.end(), perm);
  if (num_wide) *num_wide = (int)p->wide_f.size();
  if (ntasks) *ntasks = p->cs.ntasks;
  return kOk;
}

int droid_ba_plan_kx(const void* plan, int64_t* out) {
  auto* p = static_cast<const BaPlan*>(plan);
  if (!p) return fail(kInvalidArgument, "ba_plan_kx: null plan");
  for (int k = 0; k < p->K; ++k) out[k] = p->kx[k];
  return kOk;
}

// Byte offset/size of the reduced system's input tiles (the 64x64 fp64 tiles
// the assembly writes, rhs row included) inside the workspace: the contiguous
// buffer a multi-GPU caller all-reduces.  Fill tiles follow it and are zero
// before the factorisation.
int droid_ba_plan_ints_region(const void* plan, size_t* offset, size_t* bytes) {
  auto* p = static_cast<const BaPlan*>(plan);
  if (!p) return fail(kInvalidArgument, "ba_plan_ints_region: null plan");
  *offset = p->off_ints;
  *bytes = p->ints.size() * sizeof(int);
  return kOk;
}

int droid_ba_plan_system_region(const void* plan, size_t* offset, size_t* bytes) {
  auto* p = static_cast<const BaPlan*>(plan);
  if (!p) return fail(kInvalidArgument, "ba_plan_system_region: null plan");
  *offset = p->off_M;
  *bytes = (size_t)p->cs.nslots_a * kTile * 8;
  return kOk;
}

}  // extern "C"
