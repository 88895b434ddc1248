/* Declaration-only stand-in for R's <R_ext/Rdynload.h> (test infrastructure, see
 * ../Rinternals.h). */
#ifndef KMHG_RSHIM_RDYNLOAD_H
#define KMHG_RSHIM_RDYNLOAD_H

#ifdef __cplusplus
extern "C" {
#endif

typedef void *(*DL_FUNC)(void);
typedef struct {
  const char *name;
  DL_FUNC fun;
  int numArgs;
} R_CallMethodDef;
typedef R_CallMethodDef R_ExternalMethodDef;
typedef struct {
  const char *name;
  DL_FUNC fun;
  int numArgs;
  void *types;
} R_CMethodDef;
typedef R_CMethodDef R_FortranMethodDef;
typedef struct _DllInfo DllInfo;

int R_registerRoutines(DllInfo *info, const R_CMethodDef *const croutines,
                       const R_CallMethodDef *const callRoutines,
                       const R_FortranMethodDef *const fortranRoutines,
                       const R_ExternalMethodDef *const externalRoutines);

#ifdef __cplusplus
}
#endif
#endif
