/* TEST INFRASTRUCTURE (oracle) — never linked into the product.
 *
 * C restatement of scikit-image 0.18.3 segmentation.watershed for the call the Cells set uses
 * (2-D, connectivity 1, offset centre, compactness 0, watershed_line False, a mask):
 * skimage/segmentation/_watershed.py:94-227 (validate, pad by one, raveled neighbours, markers in
 * raster order) and its Cython kernel `_watershed_cy.watershed_raveled` (binary heap ordered by
 * (value, age); markers pushed first with age 0; popping a pixel pushes every unlabelled in-mask
 * 4-neighbour with a fresh age and LABELS IT AT PUSH TIME with the popped pixel's label).
 * The heap below is a plain binary min-heap on (value, age); with all pixel values distinct (the
 * elevation oracle/ws_oracle.py builds always is) the pop order is the total order on value and no
 * heap-internal tie order can matter.  Pinned by tests/golden/watershed_cases.npz (skimage 0.18.3).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  double value;
  int64_t age;
  int64_t index;
} item_t;

static int smaller(const item_t* a, const item_t* b) {
  if (a->value != b->value) return a->value < b->value;
  return a->age < b->age;
}

typedef struct {
  item_t* d;
  int64_t n, cap;
} heap_t;

static int push(heap_t* h, item_t it) {
  if (h->n == h->cap) {
    int64_t nc = h->cap ? 2 * h->cap : 1024;
    item_t* nd = (item_t*)realloc(h->d, (size_t)nc * sizeof(item_t));
    if (!nd) return -1;
    h->d = nd;
    h->cap = nc;
  }
  int64_t c = h->n++;
  h->d[c] = it;
  while (c > 0) {
    int64_t p = (c - 1) / 2;
    if (!smaller(&h->d[c], &h->d[p])) break;
    item_t t = h->d[c];
    h->d[c] = h->d[p];
    h->d[p] = t;
    c = p;
  }
  return 0;
}

static item_t pop(heap_t* h) {
  item_t top = h->d[0];
  h->d[0] = h->d[--h->n];
  int64_t i = 0;
  for (;;) {
    int64_t l = 2 * i + 1, r = l + 1, s = i;
    if (l < h->n && smaller(&h->d[l], &h->d[s])) s = l;
    if (r < h->n && smaller(&h->d[r], &h->d[s])) s = r;
    if (s == i) break;
    item_t t = h->d[i];
    h->d[i] = h->d[s];
    h->d[s] = t;
    i = s;
  }
  return top;
}

/* image float64 [H][W], markers int32 [H][W] (0 = none), mask uint8 [H][W] (NULL = all) ->
 * out int32 [H][W].  Returns 0, or -1 when out of memory. */
int watershed_c(const double* image, const int32_t* markers, const uint8_t* mask, int H, int W,
                int32_t* out) {
  const int64_t Hp = H + 2, Wp = W + 2, np_ = Hp * Wp;
  double* img = (double*)calloc((size_t)np_, sizeof(double));
  uint8_t* msk = (uint8_t*)calloc((size_t)np_, 1);
  int32_t* o = (int32_t*)calloc((size_t)np_, sizeof(int32_t));
  heap_t h = {0, 0, 0};
  int rc = -1;
  if (!img || !msk || !o) goto done;
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      const int64_t s = (int64_t)y * W + x, d = (int64_t)(y + 1) * Wp + x + 1;
      img[d] = image[s];
      msk[d] = mask ? (mask[s] != 0) : 1;
      o[d] = msk[d] ? markers[s] : 0; /* markers * mask */
    }
  {
    const int64_t nb[4] = {-Wp, -1, 1, Wp};
    for (int64_t i = 0; i < np_; ++i) /* np.flatnonzero(output): raster order, age 0 */
      if (o[i] && push(&h, (item_t){img[i], 0, i})) goto done;
    int64_t age = 1;
    while (h.n > 0) {
      const item_t e = pop(&h);
      for (int k = 0; k < 4; ++k) {
        const int64_t q = e.index + nb[k];
        if (!msk[q] || o[q]) continue;
        age += 1;
        o[q] = o[e.index];
        if (push(&h, (item_t){img[q], age, q})) goto done;
      }
    }
  }
  for (int y = 0; y < H; ++y) memcpy(out + (int64_t)y * W, o + (int64_t)(y + 1) * Wp + 1, (size_t)W * sizeof(int32_t));
  rc = 0;
done:
  free(img);
  free(msk);
  free(o);
  free(h.d);
  return rc;
}
