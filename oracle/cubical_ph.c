/*
 * ORACLE — test infrastructure only. Never linked into or called by the product path.
 *
 * CPU restatement of the sublevel-set cubical persistence that the reference computes at
 * ref:octsam/models/topological_loss.py:55-63 through
 *   torch_topological.nn.CubicalComplex(dim=2, superlevel=False)  (unpinned; absent here)
 *     -> gudhi.CubicalComplex(dimensions=x.shape, top_dimensional_cells=x.flatten())  (unpinned; absent)
 *        .persistence(); .cofaces_of_persistence_pairs()
 *
 * gudhi's published algorithm, restated:
 *   * Bitmap of (2W+1) x (2H+1) cells, position p = X + (2W+1)*Y; pixel (r,c) is the top cell
 *     X=2c+1, Y=2r+1 (gudhi's first dimension is the fastest-varying one, so the C-order flat
 *     pixel index r*W+c is exactly gudhi's top-cell index).
 *   * Lower cells take the minimum value of their top-dimensional cofaces (lower-star).
 *   * Total filtration order ("is_before_in_filtration"): (value, cell dimension, position).
 *   * Persistence pairs are those of the standard reduction for that total order (unique);
 *     intervals of zero length are discarded (min_persistence = 0).
 *   * cofaces_of_persistence_pairs maps every cell to a top-dimensional coface through
 *     get_top_dimensional_coface_of_a_cell: the FIRST coboundary cell with an equal value,
 *     recursively, where the coboundary is enumerated from the slowest axis (Y) to the fastest
 *     (X), the "-1" neighbour before the "+1" neighbour.
 *   * torch_topological pairs each essential class with argmax(x) (first maximum).
 *
 * H0 pairs come from a union-find over vertices in increasing order (elder rule); H1 pairs come
 * from the Alexander-dual union-find over pixels (plus the exterior, born at +inf) in decreasing
 * edge order. Both are checked against a brute-force Z/2 boundary-matrix reduction in
 * tests/test_oracle_ph.py.  Parity with gudhi itself is UNPINNED (gudhi is not available and the
 * reference has no tests or fixtures for this path).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  float v;
  int32_t pos;
} cell_key;

static int g_W2; /* row stride of the bitmap (2W+1), used by the comparator */

static int key_cmp(const void* a, const void* b) {
  const cell_key* x = (const cell_key*)a;
  const cell_key* y = (const cell_key*)b;
  if (x->v < y->v) return -1;
  if (x->v > y->v) return 1;
  /* equal values: all keys sorted here are of one dimension, so position decides */
  return (x->pos > y->pos) - (x->pos < y->pos);
}

typedef struct {
  int W, H, W2, H2;
  const float* x;
} bitmap;

static int cell_dim(const bitmap* b, int p) { return ((p % b->W2) & 1) + ((p / b->W2) & 1); }

static float cell_value(const bitmap* b, int p) {
  int X = p % b->W2, Y = p / b->W2;
  float best = 0.0f;
  int have = 0;
  for (int dy = -1; dy <= 1; ++dy) {
    for (int dx = -1; dx <= 1; ++dx) {
      int XX = X + dx, YY = Y + dy;
      if (!(XX & 1) || !(YY & 1)) continue;               /* top cells only */
      if (XX < 0 || YY < 0 || XX >= b->W2 || YY >= b->H2) continue;
      if ((X & 1) && dx != 0) continue;                    /* must be a coface */
      if ((Y & 1) && dy != 0) continue;
      float v = b->x[(YY >> 1) * b->W + (XX >> 1)];
      if (!have || v < best) best = v;
      have = 1;
    }
  }
  return best;
}

/* get_top_dimensional_coface_of_a_cell; returns the pixel index r*W+c */
static int top_coface(const bitmap* b, int p) {
  for (;;) {
    int X = p % b->W2, Y = p / b->W2;
    if ((X & 1) && (Y & 1)) return (Y >> 1) * b->W + (X >> 1);
    float v = cell_value(b, p);
    int next = -1;
    /* axis 1 (Y, stride W2) first, then axis 0 (X, stride 1) */
    if (!(Y & 1)) {
      if (Y > 0 && cell_value(b, p - b->W2) == v) next = p - b->W2;
      else if (Y < b->H2 - 1 && cell_value(b, p + b->W2) == v) next = p + b->W2;
    }
    if (next < 0 && !(X & 1)) {
      if (X > 0 && cell_value(b, p - 1) == v) next = p - 1;
      else if (X < b->W2 - 1 && cell_value(b, p + 1) == v) next = p + 1;
    }
    if (next < 0) return -1; /* unreachable for lower-star values */
    p = next;
  }
}

static int uf_find(int* parent, int a) {
  while (parent[a] != a) {
    parent[a] = parent[parent[a]];
    a = parent[a];
  }
  return a;
}

typedef struct {
  double pers;
  cell_key dkey; /* destroyer key */
  int c, d;      /* creator / destroyer pixel */
} pair_rec;

static int pair_cmp(const void* a, const void* b) {
  const pair_rec* x = (const pair_rec*)a;
  const pair_rec* y = (const pair_rec*)b;
  if (x->pers > y->pers) return -1;
  if (x->pers < y->pers) return 1;
  return key_cmp(&x->dkey, &y->dkey);
}

/* Returns 0 on success, 1 if a pair list overflowed max_pairs. */
int oracle_cubical_ph(const float* x, int H, int W, int max_pairs, int32_t* pairs0, int32_t* n0, int32_t* pairs1,
                      int32_t* n1, int32_t* essential) {
  bitmap b = {W, H, 2 * W + 1, 2 * H + 1, x};
  g_W2 = b.W2;
  const int ncells = b.W2 * b.H2;
  int nedges = 0;
  for (int p = 0; p < ncells; ++p)
    if (cell_dim(&b, p) == 1) ++nedges;
  cell_key* edges = (cell_key*)malloc(sizeof(cell_key) * nedges);
  int k = 0;
  for (int p = 0; p < ncells; ++p)
    if (cell_dim(&b, p) == 1) {
      edges[k].v = cell_value(&b, p);
      edges[k].pos = p;
      ++k;
    }
  qsort(edges, nedges, sizeof(cell_key), key_cmp);

  int overflow = 0;
  pair_rec* recs = (pair_rec*)malloc(sizeof(pair_rec) * (nedges + 1));

  /* ---- H0: vertices are cells (even, even); parent indexed by bitmap position */
  int* parent = (int*)malloc(sizeof(int) * ncells);
  for (int p = 0; p < ncells; ++p) parent[p] = p;
  int nr = 0;
  for (int e = 0; e < nedges; ++e) {
    int p = edges[e].pos, X = p % b.W2;
    int u, v;
    if (X & 1) { u = p - 1; v = p + 1; } else { u = p - b.W2; v = p + b.W2; }
    int ru = uf_find(parent, u), rv = uf_find(parent, v);
    if (ru == rv) continue;
    cell_key ku = {cell_value(&b, ru), ru}, kv = {cell_value(&b, rv), rv};
    int young = key_cmp(&ku, &kv) > 0 ? ru : rv;
    int old = young == ru ? rv : ru;
    parent[young] = old;
    float bv = cell_value(&b, young);
    if (edges[e].v > bv) {
      recs[nr].pers = (double)edges[e].v - (double)bv;
      recs[nr].dkey = edges[e];
      recs[nr].c = top_coface(&b, young);
      recs[nr].d = top_coface(&b, p);
      ++nr;
    }
  }
  qsort(recs, nr, sizeof(pair_rec), pair_cmp);
  if (nr > max_pairs) { overflow = 1; nr = max_pairs; }
  for (int i = 0; i < nr; ++i) { pairs0[2 * i] = recs[i].c; pairs0[2 * i + 1] = recs[i].d; }
  *n0 = nr;
  /* essential class: root of the single remaining component (the global minimum vertex) */
  int root = uf_find(parent, 0);
  essential[0] = top_coface(&b, root);
  int am = 0;
  for (int i = 1; i < W * H; ++i)
    if (x[i] > x[am]) am = i;
  essential[1] = am;

  /* ---- H1: dual union-find over pixels (index 0..W*H-1) plus exterior node W*H */
  const int EXT = W * H;
  int* par2 = parent; /* reuse */
  for (int i = 0; i <= EXT; ++i) par2[i] = i;
  nr = 0;
  for (int e = nedges - 1; e >= 0; --e) {
    int p = edges[e].pos, X = p % b.W2, Y = p / b.W2;
    int a, c;
    if (X & 1) { /* X odd, Y even: pixels above/below */
      int col = X >> 1;
      a = (Y > 0) ? ((Y >> 1) - 1) * W + col : EXT;
      c = (Y < b.H2 - 1) ? (Y >> 1) * W + col : EXT;
    } else {     /* X even, Y odd: pixels left/right */
      int row = Y >> 1;
      a = (X > 0) ? row * W + (X >> 1) - 1 : EXT;
      c = (X < b.W2 - 1) ? row * W + (X >> 1) : EXT;
    }
    int ra = uf_find(par2, a), rc = uf_find(par2, c);
    if (ra == rc) continue;
    int young, old;
    if (ra == EXT) { young = rc; old = ra; }
    else if (rc == EXT) { young = ra; old = rc; }
    else {
      int pa = (2 * (ra / W) + 1) * b.W2 + 2 * (ra % W) + 1;
      int pc = (2 * (rc / W) + 1) * b.W2 + 2 * (rc % W) + 1;
      cell_key ka = {x[ra], pa}, kc = {x[rc], pc};
      if (key_cmp(&ka, &kc) < 0) { young = ra; old = rc; } else { young = rc; old = ra; }
    }
    par2[young] = old;
    float dv = x[young];
    if (dv > edges[e].v) {
      recs[nr].pers = (double)dv - (double)edges[e].v;
      recs[nr].dkey.v = dv;
      recs[nr].dkey.pos = (2 * (young / W) + 1) * b.W2 + 2 * (young % W) + 1;
      recs[nr].c = top_coface(&b, p);
      recs[nr].d = young;
      ++nr;
    }
  }
  qsort(recs, nr, sizeof(pair_rec), pair_cmp);
  if (nr > max_pairs) { overflow = 1; nr = max_pairs; }
  for (int i = 0; i < nr; ++i) { pairs1[2 * i] = recs[i].c; pairs1[2 * i + 1] = recs[i].d; }
  *n1 = nr;

  free(parent);
  free(recs);
  free(edges);
  return overflow;
}
