/* oracle/r1cs_shape.inc.c — the constraint STRUCTURE of the restated circuit, and circom-shaped signal maps
 * derived from it. Included by r1cs_check.c.
 *
 * TOOL / TEST INFRASTRUCTURE ONLY: used by tools/gen_shape_maps.py (which writes the committed maps under
 * passport-zk-circuits_amd/data/shape/) and by tests/; the shipped library never links it.
 *
 * What a prover reads is the witness circom writes after simplification: `--O2` in the main flow
 * (circuits/scripts/compile-circuit.sh:34, read by circuits/scripts/prove.sh:27), `--O1` in the library flow
 * (circuits/lib/circuits/scripts/compile-circuit.sh:34). circom documents them as
 *   --O1: signal = signal constraints merge the two signals, signal = constant constraints remove the signal;
 *   --O2: in addition, every linear constraint substitutes one of its signals away.
 * Main's inputs and outputs are never removed. circom is absent here and the snapshot does not compile
 * (SURVEY.md §8c), so the structure is read off the restated constraints (r1cs_check.c) instead of a .r1cs:
 *
 *   ck_structure() walks the circuit four times over synthetic witnesses w0, w0 + d, w0 + 2d, w0 + d' (random
 *   field elements, w[0] = 1; the walk's control flow never depends on values). Each constraint records the
 *   signals it reads (its support) and its residual r = lhs - rhs. r is affine in the witness iff
 *   r(w0) - 2 r(w0 + d) + r(w0 + 2d) = 0 (a quadratic term survives the second difference for random d, except
 *   with probability ~1/p). A linear constraint over one signal fixes it to a constant; one over two signals
 *   x, y is a copy iff r = s (x - y), s = +-1, at all three points w0, d, d'.
 *
 *   ck_shape_map() turns that into a witness map the way the documented rules read: copies merge (union-find,
 *   the lowest signal index represents its class), constants remove, and at level 2 each remaining linear
 *   constraint removes the highest-indexed signal class of its support not yet removed, and signals no
 *   constraint reads are dropped. WHICH signal circom substitutes, its elimination order and whether it merges
 *   or removes a copy are circom internals: the maps are shaped like circom's (the same classes of signals
 *   survive: bits, products, inverses; sums, copies and constants go), their exact contents are
 *   PARITY UNPINNED.
 */

static void tr_grow(void **p, uint64_t *cap, uint64_t need, size_t el) {
  if (need <= *cap || (TR && TR->nomem)) return;
  uint64_t c = *cap ? *cap : 1024;
  while (c < need) c *= 2;
  void *q = realloc(*p, c * el);
  if (!q) { TR->nomem = 1; return; }
  *p = q;
  *cap = c;
}
static void tr_read(size_t i) {
  tr_grow((void **)&TR->sig, &TR->cap_sig, TR->n_sig + 1, sizeof(uint32_t));
  if (TR->nomem) return;
  TR->sig[TR->n_sig++] = (uint32_t)i;
}
static void tr_cons(fr_t residual) {
  tr_grow((void **)&TR->off, &TR->cap_cons, TR->n_cons + 2, sizeof(uint64_t));
  tr_grow((void **)&TR->res, &TR->cap_res, TR->n_cons + 2, sizeof(fr_t));
  if (TR->nomem) return;
  TR->res[TR->n_cons] = residual;
  TR->off[++TR->n_cons] = TR->n_sig;
}

/* the synthetic witness values: a counter-based generator, so each run regenerates its vector */
static uint64_t sh_mix(uint64_t z) {
  z += 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
static fr_t sh_rand(uint64_t seed, uint64_t stream, uint64_t i) {
  fr_t r;
  for (int k = 0; k < 4; k++) r.l[k] = sh_mix(seed ^ sh_mix(stream * 0x100000001b3ULL + 4 * i + k));
  r.l[3] &= 0x0fffffffffffffffULL;  /* < 2^252 < p */
  return r;
}

enum { CK_CIRC_REGISTER = 0, CK_CIRC_QUERY = 1, CK_CIRC_SHA256 = 2, CK_CIRC_POSEIDON = 3 };

static int shape_walk(ck_t *c, int circuit, int arg, const ck_params *P, size_t *walked) {
  switch (circuit) {
    case CK_CIRC_REGISTER:
      if (!pos_loaded) return -1;
      if (P->sig >= 20) {
        if (ec_curve_of(P->sig) < 0) return -2;
        CV = &EC[ec_curve_of(P->sig)];
        EK = CV->nl; EB = CV->cs;
        if (!CV->gpow) return -3;
      }
      *walked = 1 + ck_builder(c, 1, P);
      return 0;
    case CK_CIRC_QUERY:
      if (!pos_loaded) return -1;
      CKQ_TD1 = arg != 0;
      *walked = 1 + ck_queryid(c, 1);
      return 0;
    case CK_CIRC_SHA256: *walked = 1 + ck_sha2chunks(c, 1, arg, 256); return 0;
    case CK_CIRC_POSEIDON:
      if (!pos_loaded) return -1;
      *walked = 1 + ck_poseidon(c, 1, arg);
      return 0;
  }
  return -2;
}

typedef struct {
  uint64_t n_cons;  /* constraints of the walk */
  uint64_t n_sup;   /* entries of sup */
  uint8_t *cls;     /* per constraint: CK_QUAD / CK_LIN / CK_COPY / CK_CONST */
  uint64_t *off;    /* n_cons + 1: the support of constraint j is sup[off[j] .. off[j + 1]) */
  uint32_t *sup;    /* its distinct signals, ascending; the constant signal 0 is not listed */
} ck_struct;
enum { CK_QUAD = 0, CK_LIN = 1, CK_COPY = 2, CK_CONST = 3 };

static int cmp_u32(const void *a, const void *b) {
  uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
  return x < y ? -1 : x > y;
}

void ck_struct_free(ck_struct *s) {
  free(s->cls); free(s->off); free(s->sup);
  memset(s, 0, sizeof *s);
}

/* n: the circuit's O0 witness size. Returns 0, or < 0: -1 constants not loaded, -2 bad circuit, -4 the walk does
 * not cover n, -5 out of memory, -6 the walk's reads differ between runs (value-dependent control flow) */
int ck_structure(int circuit, int arg, const ck_params *P, size_t n, uint64_t seed, ck_struct *out) {
  ck_init();
  memset(out, 0, sizeof *out);
  fr_t *w = malloc(n * sizeof(fr_t));
  ck_tr_t tr[4];
  memset(tr, 0, sizeof tr);
  int rc = w ? 0 : -5;
  /* run k: w0 + m_k d + e_k d' with (m, e) = (0,0), (1,0), (2,0), (0,1) */
  static const int M[4] = {0, 1, 2, 0}, E[4] = {0, 0, 0, 1};
  for (int k = 0; k < 4 && !rc; k++) {
    for (size_t i = 0; i < n; i++) {
      fr_t v = sh_rand(seed, 0, i);
      if (M[k]) { fr_t d = sh_rand(seed, 1, i); v = fr_add(v, d); if (M[k] == 2) v = fr_add(v, d); }
      if (E[k]) v = fr_add(v, sh_rand(seed, 2, i));
      w[i] = v;
    }
    w[0] = fr_u64(1);
    ck_t c = ck_begin((const uint8_t *)w, n);
    size_t walked = 0;
    TR = &tr[k];
    tr_cons(fr_zero());  /* allocate off[0] */
    tr[k].n_cons = 0;
    tr[k].off[0] = 0;
    rc = shape_walk(&c, circuit, arg, P, &walked);
    TR = NULL;
    free(c.cov);
    if (!rc && (walked != n || c.oob)) rc = -4;
    if (!rc && tr[k].nomem) rc = -5;
    if (!rc && k > 0 && (tr[k].n_cons != tr[0].n_cons || tr[k].n_sig != tr[0].n_sig ||
                         memcmp(tr[k].sig, tr[0].sig, tr[0].n_sig * sizeof(uint32_t)))) rc = -6;
    if (k >= 1) { free(tr[k].sig); tr[k].sig = NULL; free(tr[k].off); tr[k].off = NULL; }
  }
  free(w);
  const uint64_t nc = tr[0].n_cons;
  if (!rc) {
    out->n_cons = nc;
    out->cls = calloc(nc ? nc : 1, 1);
    out->off = malloc((nc + 1) * sizeof(uint64_t));
    out->sup = malloc((tr[0].n_sig ? tr[0].n_sig : 1) * sizeof(uint32_t));
    if (!out->cls || !out->off || !out->sup) rc = -5;
  }
  if (!rc) {
    uint64_t ns = 0;
    out->off[0] = 0;
    for (uint64_t j = 0; j < nc; j++) {
      /* support: the distinct signals read, without the constant 0 */
      uint64_t a = tr[0].off[j], b = tr[0].off[j + 1], s0 = ns;
      for (uint64_t t = a; t < b; t++)
        if (tr[0].sig[t]) out->sup[ns++] = tr[0].sig[t];
      qsort(out->sup + s0, ns - s0, sizeof(uint32_t), cmp_u32);
      uint64_t u = s0;
      for (uint64_t t = s0; t < ns; t++)
        if (t == s0 || out->sup[t] != out->sup[u - 1]) out->sup[u++] = out->sup[t];
      ns = u;
      out->off[j + 1] = ns;
      const fr_t r0 = tr[0].res[j], r1 = tr[1].res[j], r2 = tr[2].res[j], r3 = tr[3].res[j];
      /* second difference along d */
      if (!fr_is_zero(fr_add(fr_sub(r0, fr_add(r1, r1)), r2))) { out->cls[j] = CK_QUAD; continue; }
      const uint64_t k = ns - s0;
      const fr_t d1 = fr_sub(r1, r0), d3 = fr_sub(r3, r0);
      out->cls[j] = CK_LIN;
      if (k == 1 && (!fr_is_zero(d1) || !fr_is_zero(d3))) out->cls[j] = CK_CONST;
      if (k == 2) {
        const uint32_t x = out->sup[s0], y = out->sup[s0 + 1];
        const fr_t vx = sh_rand(seed, 0, x), vy = sh_rand(seed, 0, y);
        const fr_t e0 = fr_sub(vx, vy), e1 = fr_sub(sh_rand(seed, 1, x), sh_rand(seed, 1, y)),
                   e3 = fr_sub(sh_rand(seed, 2, x), sh_rand(seed, 2, y));
        const int pos = fr_eq(r0, e0) && fr_eq(d1, e1) && fr_eq(d3, e3);
        const int neg = fr_eq(r0, fr_neg(e0)) && fr_eq(d1, fr_neg(e1)) && fr_eq(d3, fr_neg(e3));
        if (pos || neg) out->cls[j] = CK_COPY;
      }
    }
    out->n_sup = ns;
  }
  for (int k = 0; k < 4; k++) { free(tr[k].sig); free(tr[k].off); free(tr[k].res); }
  if (rc) ck_struct_free(out);
  return rc;
}

static uint32_t uf_find(uint32_t *par, uint32_t x) {
  while (par[x] != x) { par[x] = par[par[x]]; x = par[x]; }
  return x;
}

/* level 1 (--O1-shaped) or 2 (--O2-shaped) witness map over the n O0 signals: wit[s] = witness index of signal s,
 * -1 = removed; wit[0] = 0. Signals 1 .. n_protect - 1 (main's outputs and inputs) are never removed or merged
 * away. Witness indices increase with the lowest signal of each class (a monotone map: pzk_instance_create_mapped
 * emits it directly). Returns the witness size (the number of indices), or < 0. */
int64_t ck_shape_map(const ck_struct *st, size_t n, size_t n_protect, int level, int32_t *wit) {
  uint32_t *par = malloc(n * sizeof(uint32_t));
  uint8_t *fl = calloc(n, 1);  /* per class root: 1 holds a protected signal, 2 constant, 4 removed; 8 = read */
  if (!par || !fl) { free(par); free(fl); return -5; }
  enum { F_PROT = 1, F_CONST = 2, F_GONE = 4, F_READ = 8 };
  for (size_t i = 0; i < n; i++) par[i] = (uint32_t)i;
  for (size_t i = 0; i < n_protect && i < n; i++) fl[i] |= F_PROT;
  for (uint64_t j = 0; j < st->n_cons; j++)
    for (uint64_t t = st->off[j]; t < st->off[j + 1]; t++) fl[st->sup[t]] |= F_READ;
  /* copies: merge the two classes (lower root wins) unless both hold a protected signal */
  for (uint64_t j = 0; j < st->n_cons; j++) {
    if (st->cls[j] != CK_COPY) continue;
    uint32_t a = uf_find(par, st->sup[st->off[j]]), b = uf_find(par, st->sup[st->off[j] + 1]);
    if (a == b || ((fl[a] & F_PROT) && (fl[b] & F_PROT))) continue;
    if (b < a) { uint32_t t = a; a = b; b = t; }
    par[b] = a;
    fl[a] |= fl[b] & (F_PROT | F_CONST);
  }
  /* constants: the class is fixed (it stays only through a protected member) */
  for (uint64_t j = 0; j < st->n_cons; j++)
    if (st->cls[j] == CK_CONST) fl[uf_find(par, st->sup[st->off[j]])] |= F_CONST;
  if (level >= 2) {
    /* every other linear constraint substitutes one class away: the highest one still free */
    for (uint64_t j = 0; j < st->n_cons; j++) {
      if (st->cls[j] != CK_LIN) continue;
      uint32_t best = 0;
      int found = 0;
      for (uint64_t t = st->off[j]; t < st->off[j + 1]; t++) {
        uint32_t r = uf_find(par, st->sup[t]);
        if (fl[r] & (F_PROT | F_CONST | F_GONE)) continue;
        if (!found || r > best) { best = r; found = 1; }
      }
      if (found) fl[best] |= F_GONE;
    }
  }
  int64_t next = 1;
  wit[0] = 0;
  for (size_t s = 1; s < n; s++) {
    const uint32_t r = uf_find(par, (uint32_t)s);
    const int prot = s < n_protect;
    if (prot) { wit[s] = (int32_t)next++; continue; }
    if ((fl[r] & (F_CONST | F_GONE)) && !(fl[r] & F_PROT)) { wit[s] = -1; continue; }
    if (level >= 2 && r == s && !(fl[s] & F_READ)) { wit[s] = -1; continue; }  /* read by no constraint */
    if (r == s) { wit[s] = (int32_t)next++; continue; }
    wit[s] = wit[r];  /* r < s: assigned already (or -1 with its class) */
  }
  free(par); free(fl);
  return next;
}
