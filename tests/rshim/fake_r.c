/* fake_r.c -- a tiny R runtime for driving the R glue's .Call entry points from the tests
 * (test infrastructure only; R itself is not installed in this image).
 *
 * It implements the R API subset declared in the headers beside it with R's semantics where the glue
 * depends on them: error() unwinds to the caller of the .Call (longjmp, like R's error
 * handling), PROTECT/UNPROTECT are counted so an unbalanced entry point is reported,
 * allocMatrix checks its dimensions, external pointers carry tag, address and finaliser, and
 * R_registerRoutines records the registration table.  Objects live until fr_reset().  The
 * glue and this file are linked into one shared library (tests/test_r_glue.py), which the tests
 * load with ctypes: fr_* below build arguments, make calls by registered name, and read
 * results. */
#include <setjmp.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "R.h"
#include "Rinternals.h"
#include "R_ext/Rdynload.h"

struct SEXPREC {
  SEXPTYPE type;
  R_xlen_t n;
  int nrow, ncol;              /* matrices: nrow x ncol, else -1 */
  int *ip;
  double *dp;
  SEXP *vp;                    /* STRSXP / VECSXP elements */
  char *cp;                    /* CHARSXP */
  void *addr;                  /* EXTPTRSXP */
  SEXP tag, prot, names;
  R_CFinalizer_t fin;
  int fin_onexit;
  struct SEXPREC *next;        /* every object, for fr_reset / finalisers */
};

static struct SEXPREC nil_obj = {NILSXP, 0, -1, -1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
static struct SEXPREC names_sym = {NILSXP, 0, -1, -1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
SEXP R_NilValue = &nil_obj;
SEXP R_NamesSymbol = &names_sym;

static struct SEXPREC *all_objs;
static void **allocs;
static size_t n_allocs, cap_allocs;
static int protect_depth;
static jmp_buf *err_jmp;
static char err_msg[4096], warn_msg[4096];
static int n_warnings;

static void *arena(size_t bytes) {
  void *p = calloc(1, bytes ? bytes : 1);
  if (!p) abort();
  if (n_allocs == cap_allocs) {
    cap_allocs = cap_allocs ? 2 * cap_allocs : 256;
    allocs = (void **)realloc(allocs, cap_allocs * sizeof(void *));
    if (!allocs) abort();
  }
  allocs[n_allocs++] = p;
  return p;
}

static SEXP new_obj(SEXPTYPE t, R_xlen_t n) {
  SEXP s = (SEXP)arena(sizeof(struct SEXPREC));
  s->type = t;
  s->n = n;
  s->nrow = s->ncol = -1;
  s->tag = s->prot = s->names = R_NilValue;
  s->next = all_objs;
  all_objs = s;
  return s;
}

/* ---- the R API subset (Rinternals.h / R.h / Rdynload.h) ---- */
void Rf_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(err_msg, sizeof err_msg, fmt, ap);
  va_end(ap);
  if (!err_jmp) {
    fprintf(stderr, "fake_r: error() outside a call: %s\n", err_msg);
    abort();
  }
  longjmp(*err_jmp, 1);
}
void Rf_warning(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(warn_msg, sizeof warn_msg, fmt, ap);
  va_end(ap);
  ++n_warnings;
}
void Rprintf(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vprintf(fmt, ap);
  va_end(ap);
}
char *R_alloc(size_t nelem, int eltsize) { return (char *)arena(nelem * (size_t)eltsize); }

int TYPEOF(SEXP x) { return (int)x->type; }
R_len_t Rf_length(SEXP x) { return x == R_NilValue ? 0 : (R_len_t)x->n; }
R_xlen_t XLENGTH(SEXP x) { return x == R_NilValue ? 0 : x->n; }
int *INTEGER(SEXP x) {
  if (x->type != INTSXP) Rf_error("INTEGER() can only be applied to a 'integer'");
  return x->ip;
}
double *REAL(SEXP x) {
  if (x->type != REALSXP) Rf_error("REAL() can only be applied to a 'numeric'");
  return x->dp;
}
const char *R_CHAR(SEXP x) {
  if (x->type != CHARSXP) Rf_error("CHAR() can only be applied to a 'CHARSXP'");
  return x->cp;
}
SEXP STRING_ELT(SEXP x, R_xlen_t i) {
  if (x->type != STRSXP || i < 0 || i >= x->n) Rf_error("STRING_ELT out of range");
  return x->vp[i];
}
void SET_STRING_ELT(SEXP x, R_xlen_t i, SEXP v) {
  if (x->type != STRSXP || i < 0 || i >= x->n || v->type != CHARSXP)
    Rf_error("SET_STRING_ELT misuse");
  x->vp[i] = v;
}
SEXP VECTOR_ELT(SEXP x, R_xlen_t i) {
  if (x->type != VECSXP || i < 0 || i >= x->n) Rf_error("VECTOR_ELT out of range");
  return x->vp[i];
}
SEXP SET_VECTOR_ELT(SEXP x, R_xlen_t i, SEXP v) {
  if (x->type != VECSXP || i < 0 || i >= x->n) Rf_error("SET_VECTOR_ELT out of range");
  x->vp[i] = v;
  return v;
}
SEXP Rf_mkChar(const char *s) {
  SEXP c = new_obj(CHARSXP, (R_xlen_t)strlen(s));
  c->cp = (char *)arena(strlen(s) + 1);
  memcpy(c->cp, s, strlen(s) + 1);
  return c;
}
SEXP Rf_allocVector(SEXPTYPE t, R_xlen_t n) {
  if (n < 0) Rf_error("negative length vectors are not allowed");
  SEXP s = new_obj(t, n);
  switch (t) {
    case INTSXP: s->ip = (int *)arena((size_t)n * sizeof(int)); break;
    case REALSXP: s->dp = (double *)arena((size_t)n * sizeof(double)); break;
    case STRSXP: {
      s->vp = (SEXP *)arena((size_t)n * sizeof(SEXP));
      SEXP blank = Rf_mkChar("");
      for (R_xlen_t i = 0; i < n; ++i) s->vp[i] = blank;
      break;
    }
    case VECSXP:
      s->vp = (SEXP *)arena((size_t)n * sizeof(SEXP));
      for (R_xlen_t i = 0; i < n; ++i) s->vp[i] = R_NilValue;
      break;
    default: Rf_error("allocVector: type %u not supported by fake_r", t);
  }
  return s;
}
SEXP Rf_allocMatrix(SEXPTYPE t, int nrow, int ncol) {
  if (nrow < 0 || ncol < 0) Rf_error("negative extents to matrix");
  SEXP s = Rf_allocVector(t, (R_xlen_t)nrow * ncol);
  s->nrow = nrow;
  s->ncol = ncol;
  return s;
}
SEXP Rf_protect(SEXP s) {
  ++protect_depth;
  return s;
}
void Rf_unprotect(int n) { protect_depth -= n; }
int Rf_asInteger(SEXP x) {
  if (x->type == INTSXP && x->n >= 1) return x->ip[0];
  if (x->type == REALSXP && x->n >= 1) return (int)x->dp[0];
  return INT32_MIN;   /* NA_INTEGER */
}
SEXP Rf_setAttrib(SEXP vec, SEXP name, SEXP val) {
  if (name == R_NamesSymbol) vec->names = val;
  return val;
}
void *R_ExternalPtrAddr(SEXP s) { return s->type == EXTPTRSXP ? s->addr : NULL; }
SEXP R_ExternalPtrTag(SEXP s) { return s->tag; }
SEXP R_MakeExternalPtr(void *p, SEXP tag, SEXP prot) {
  SEXP s = new_obj(EXTPTRSXP, 1);
  s->addr = p;
  s->tag = tag;
  s->prot = prot;
  return s;
}
void R_RegisterCFinalizerEx(SEXP s, R_CFinalizer_t fun, Rboolean onexit) {
  s->fin = fun;
  s->fin_onexit = (int)onexit;
}
void R_ClearExternalPtr(SEXP s) { s->addr = NULL; }

#define MAX_ROUTINES 64
static R_CallMethodDef routines[MAX_ROUTINES];
static int n_routines;
int R_registerRoutines(DllInfo *info, const R_CMethodDef *const c, const R_CallMethodDef *const call,
                       const R_FortranMethodDef *const f, const R_ExternalMethodDef *const e) {
  (void)info; (void)c; (void)f; (void)e;
  n_routines = 0;
  for (const R_CallMethodDef *r = call; r && r->name && n_routines < MAX_ROUTINES; ++r)
    routines[n_routines++] = *r;
  return 1;
}

/* ---- the test driver's side (ctypes) ---- */
void R_init_kmer_hash(DllInfo *info);   /* the glue's registration entry */

int fr_init(void) {
  R_init_kmer_hash(NULL);
  return n_routines;
}
const char *fr_routine(int i, int *nargs) {
  if (i < 0 || i >= n_routines) return NULL;
  *nargs = routines[i].numArgs;
  return routines[i].name;
}
SEXP fr_nil(void) { return R_NilValue; }
SEXP fr_str(const char *const *v, const int64_t *lens, int64_t n) {
  SEXP s = Rf_allocVector(STRSXP, (R_xlen_t)n);
  for (int64_t i = 0; i < n; ++i) {
    SEXP c = new_obj(CHARSXP, (R_xlen_t)lens[i]);
    c->cp = (char *)arena((size_t)lens[i] + 1);
    memcpy(c->cp, v[i], (size_t)lens[i]);
    s->vp[i] = c;
  }
  return s;
}
SEXP fr_int(const int *v, int64_t n) {
  SEXP s = Rf_allocVector(INTSXP, (R_xlen_t)n);
  if (n) memcpy(s->ip, v, (size_t)n * sizeof(int));
  return s;
}
SEXP fr_real(const double *v, int64_t n) {
  SEXP s = Rf_allocVector(REALSXP, (R_xlen_t)n);
  if (n) memcpy(s->dp, v, (size_t)n * sizeof(double));
  return s;
}
SEXP fr_extptr(void *addr, const char *tag) {
  SEXP t = R_NilValue;
  if (tag) {
    t = Rf_allocVector(STRSXP, 1);
    t->vp[0] = Rf_mkChar(tag);
  }
  return R_MakeExternalPtr(addr, t, R_NilValue);
}
int fr_type(SEXP s) { return (int)s->type; }
int64_t fr_len(SEXP s) { return (int64_t)XLENGTH(s); }
int fr_nrow(SEXP s) { return s->nrow; }
int fr_ncol(SEXP s) { return s->ncol; }
int *fr_ints(SEXP s) { return s->type == INTSXP ? s->ip : NULL; }
double *fr_reals(SEXP s) { return s->type == REALSXP ? s->dp : NULL; }
SEXP fr_elt(SEXP s, int64_t i) { return (s->type == VECSXP || s->type == STRSXP) ? s->vp[i] : R_NilValue; }
const char *fr_chars(SEXP s) { return s->type == CHARSXP ? s->cp : NULL; }
SEXP fr_names(SEXP s) { return s->names; }
void *fr_addr(SEXP s) { return R_ExternalPtrAddr(s); }
const char *fr_tag(SEXP s) {
  return (s->type == EXTPTRSXP && s->tag->type == STRSXP && s->tag->n == 1) ? s->tag->vp[0]->cp : NULL;
}
int fr_has_finalizer(SEXP s) { return s->fin != NULL && s->fin_onexit; }
const char *fr_last_error(void) { return err_msg; }
const char *fr_last_warning(void) { return warn_msg; }
int fr_warnings(void) { return n_warnings; }

/* .Call(name, args...) -> 0 and *out = result, 1 on error() (message: fr_last_error), 2 for an
 * unknown name or wrong arity, 3 if the entry point returned with PROTECT/UNPROTECT unbalanced */
int fr_call(const char *name, int nargs, SEXP *args, SEXP *out) {
  DL_FUNC found = NULL;
  for (int i = 0; i < n_routines; ++i)
    if (!strcmp(routines[i].name, name)) {
      if (routines[i].numArgs != nargs) return 2;
      found = routines[i].fun;
    }
  if (!found) return 2;
  DL_FUNC volatile f = found;
  jmp_buf jb;
  jmp_buf *prev = err_jmp;
  err_jmp = &jb;
  const int depth0 = protect_depth;
  err_msg[0] = 0;
  if (setjmp(jb)) {
    err_jmp = prev;
    protect_depth = depth0;    /* R resets the protect stack on error */
    return 1;
  }
  SEXP r = R_NilValue;
  switch (nargs) {
    case 1: r = ((SEXP(*)(SEXP))(void (*)(void))f)(args[0]); break;
    case 2: r = ((SEXP(*)(SEXP, SEXP))(void (*)(void))f)(args[0], args[1]); break;
    case 3: r = ((SEXP(*)(SEXP, SEXP, SEXP))(void (*)(void))f)(args[0], args[1], args[2]); break;
    case 5: r = ((SEXP(*)(SEXP, SEXP, SEXP, SEXP, SEXP))(void (*)(void))f)(args[0], args[1], args[2], args[3], args[4]); break;
    default: err_jmp = prev; return 2;
  }
  err_jmp = prev;
  *out = r;
  return protect_depth == depth0 ? 0 : 3;
}

/* run one external pointer's finaliser (R's gc / onexit) */
int fr_finalize(SEXP s) {
  if (s->type != EXTPTRSXP || !s->fin) return 0;
  R_CFinalizer_t f = s->fin;
  s->fin = NULL;
  f(s);
  return 1;
}

/* finalise every external pointer, then free every object */
void fr_reset(void) {
  for (struct SEXPREC *s = all_objs; s; s = s->next)
    if (s->type == EXTPTRSXP && s->fin) fr_finalize(s);
  for (size_t i = 0; i < n_allocs; ++i) free(allocs[i]);
  n_allocs = 0;
  all_objs = NULL;
  n_warnings = 0;
}
