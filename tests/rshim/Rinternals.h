/* Declaration-only stand-in for R's <Rinternals.h> (test infrastructure; R is not installed
 * in this image).  It declares the subset of R's public C API that
 * kmer_hasher_amd/R/kmer_hash_glue.c uses, with R's own signatures, type codes and Rf_ remaps,
 * so that the glue is type-checked (gcc -fsyntax-only -Wall -Werror) and can be linked against
 * tests/rshim/fake_r.c, a tiny runtime that lets the tests drive the glue's .Call entry points.
 * Nothing here is R's code: only the API's names and types. */
#ifndef KMHG_RSHIM_RINTERNALS_H
#define KMHG_RSHIM_RINTERNALS_H
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct SEXPREC *SEXP;
typedef unsigned int SEXPTYPE;
typedef int R_len_t;
typedef ptrdiff_t R_xlen_t;
typedef enum { FALSE = 0, TRUE } Rboolean;

#define NILSXP 0
#define CHARSXP 9
#define INTSXP 13
#define REALSXP 14
#define STRSXP 16
#define VECSXP 19
#define EXTPTRSXP 22

extern SEXP R_NilValue;
extern SEXP R_NamesSymbol;

int TYPEOF(SEXP x);
R_len_t Rf_length(SEXP x);
R_xlen_t XLENGTH(SEXP x);
int *INTEGER(SEXP x);
double *REAL(SEXP x);
const char *R_CHAR(SEXP x);
SEXP STRING_ELT(SEXP x, R_xlen_t i);
void SET_STRING_ELT(SEXP x, R_xlen_t i, SEXP v);
SEXP VECTOR_ELT(SEXP x, R_xlen_t i);
SEXP SET_VECTOR_ELT(SEXP x, R_xlen_t i, SEXP v);
SEXP Rf_allocVector(SEXPTYPE t, R_xlen_t n);
SEXP Rf_allocMatrix(SEXPTYPE t, int nrow, int ncol);
SEXP Rf_mkChar(const char *s);
SEXP Rf_protect(SEXP s);
void Rf_unprotect(int n);
int Rf_asInteger(SEXP x);
SEXP Rf_setAttrib(SEXP vec, SEXP name, SEXP val);

typedef void (*R_CFinalizer_t)(SEXP);
void *R_ExternalPtrAddr(SEXP s);
SEXP R_ExternalPtrTag(SEXP s);
SEXP R_MakeExternalPtr(void *p, SEXP tag, SEXP prot);
void R_RegisterCFinalizerEx(SEXP s, R_CFinalizer_t fun, Rboolean onexit);
void R_ClearExternalPtr(SEXP s);

#define CHAR(x) R_CHAR(x)
#define PROTECT(s) Rf_protect(s)
#define UNPROTECT(n) Rf_unprotect(n)
#define length Rf_length
#define allocVector Rf_allocVector
#define allocMatrix Rf_allocMatrix
#define mkChar Rf_mkChar
#define asInteger Rf_asInteger
#define setAttrib Rf_setAttrib

#ifdef __cplusplus
}
#endif
#endif
