/* Declaration-only stand-in for R's <R.h> (test infrastructure, see Rinternals.h here). */
#ifndef KMHG_RSHIM_R_H
#define KMHG_RSHIM_R_H
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

char *R_alloc(size_t nelem, int eltsize);
void Rf_error(const char *fmt, ...) __attribute__((noreturn, format(printf, 1, 2)));
void Rf_warning(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
void Rprintf(const char *fmt, ...) __attribute__((format(printf, 1, 2)));

#define error Rf_error
#define warning Rf_warning

#ifdef __cplusplus
}
#endif
#endif
