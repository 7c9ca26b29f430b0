/*
 * mexshim.c -- test shim of the MEX/mx* API (mex.h, matrix.h; NOT MATLAB).
 *
 * Built with matlab/mpcekf_mex.c into tests/mex/_build/libmpcekf_mexshim.so
 * (__graft_entry__.build, tests/mex/Makefile).  tests/mexshim.py builds mxArrays
 * from numpy arrays (column-major, MATLAB class ids) and calls the gateway's
 * mexFunction through shim_call, which turns mexErrMsgIdAndTxt into an error
 * return (setjmp/longjmp, as MATLAB unwinds a MEX error) and frees the call's
 * mxMalloc'd memory afterwards, as MATLAB does when a MEX function returns.
 */
#define _POSIX_C_SOURCE 200809L
#include <setjmp.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mex.h"

#define MAXDIM 8

struct mxArray_tag {
  mxClassID cls;
  int complex;
  mwSize nd;
  mwSize dims[MAXDIM];
  void *data;                 /* numeric / char payload, column-major */
  int nfields;                /* struct arrays (1 x 1 only) */
  char **names;
  mxArray **values;
};

static size_t esize(mxClassID c) {
  switch (c) {
    case mxDOUBLE_CLASS: case mxINT64_CLASS: case mxUINT64_CLASS: return 8;
    case mxSINGLE_CLASS: case mxINT32_CLASS: case mxUINT32_CLASS: return 4;
    case mxINT16_CLASS: case mxUINT16_CLASS: return 2;
    case mxINT8_CLASS: case mxUINT8_CLASS: case mxLOGICAL_CLASS: case mxCHAR_CLASS: return 1;
    default: return 0;
  }
}

/* ---- per-call bookkeeping ------------------------------------------------ */
typedef struct Blk {
  struct Blk *next;
} Blk;
static Blk *g_blocks;      /* mxMalloc'd during the current call */
static jmp_buf *g_jmp;     /* set while a call runs */
static char g_msg[1024];

void *mxMalloc(size_t n) {
  Blk *b = (Blk *)calloc(1, sizeof(Blk) + n + 16);
  if (!b) return NULL;
  b->next = g_blocks;
  g_blocks = b;
  return (char *)b + sizeof(Blk);
}

void mxFree(void *p) {
  if (!p) return;
  for (Blk **pp = &g_blocks; *pp; pp = &(*pp)->next)
    if ((char *)*pp + sizeof(Blk) == (char *)p) {
      Blk *b = *pp;
      *pp = b->next;
      free(b);
      return;
    }
}

static void free_blocks(void) {
  while (g_blocks) {
    Blk *b = g_blocks;
    g_blocks = b->next;
    free(b);
  }
}

void mexErrMsgIdAndTxt(const char *id, const char *fmt, ...) {
  va_list ap;
  int k = snprintf(g_msg, sizeof g_msg, "%s: ", id ? id : "");
  va_start(ap, fmt);
  vsnprintf(g_msg + k, sizeof g_msg - (size_t)k, fmt, ap);
  va_end(ap);
  if (g_jmp) longjmp(*g_jmp, 1);
  fprintf(stderr, "mexshim: error outside a call: %s\n", g_msg);
  abort();
}

/* ---- arrays -------------------------------------------------------------- */
static mxArray *make(mxClassID cls, int cplx, mwSize nd, const mwSize *dims) {
  mxArray *a = (mxArray *)calloc(1, sizeof(mxArray));
  a->cls = cls;
  a->complex = cplx;
  a->nd = nd < 2 ? 2 : nd;
  a->dims[0] = a->dims[1] = 1;
  for (mwSize i = 0; i < nd && i < MAXDIM; ++i) a->dims[i] = dims[i];
  size_t n = 1;
  for (mwSize i = 0; i < a->nd; ++i) n *= a->dims[i];
  const size_t es = esize(cls) * (cplx ? 2 : 1);
  if (es) a->data = calloc(n ? n : 1, es);
  return a;
}

mxArray *mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity c) {
  mwSize d[2] = {m, n};
  return make(mxDOUBLE_CLASS, c == mxCOMPLEX, 2, d);
}
mxArray *mxCreateDoubleScalar(double v) {
  mxArray *a = mxCreateDoubleMatrix(1, 1, mxREAL);
  *(double *)a->data = v;
  return a;
}
mxArray *mxCreateNumericMatrix(mwSize m, mwSize n, mxClassID cls, mxComplexity c) {
  mwSize d[2] = {m, n};
  return make(cls, c == mxCOMPLEX, 2, d);
}
mxArray *mxCreateStructMatrix(mwSize m, mwSize n, int nfields, const char **names) {
  if (m != 1 || n != 1) mexErrMsgIdAndTxt("mexshim:unsupported", "struct arrays other than 1 x 1");
  mwSize d[2] = {1, 1};
  mxArray *a = make(mxSTRUCT_CLASS, 0, 2, d);
  a->nfields = nfields;
  a->names = (char **)calloc((size_t)nfields + 1, sizeof(char *));
  a->values = (mxArray **)calloc((size_t)nfields + 1, sizeof(mxArray *));
  for (int i = 0; i < nfields; ++i) a->names[i] = strdup(names[i]);
  return a;
}
void mxDestroyArray(mxArray *a) {
  if (!a) return;
  for (int i = 0; i < a->nfields; ++i) {
    free(a->names[i]);
    mxDestroyArray(a->values[i]);
  }
  free(a->names);
  free(a->values);
  free(a->data);
  free(a);
}

bool mxIsDouble(const mxArray *a) { return a && a->cls == mxDOUBLE_CLASS; }
bool mxIsInt32(const mxArray *a) { return a && a->cls == mxINT32_CLASS; }
bool mxIsUint64(const mxArray *a) { return a && a->cls == mxUINT64_CLASS; }
bool mxIsNumeric(const mxArray *a) { return a && a->cls >= mxDOUBLE_CLASS && a->cls <= mxUINT64_CLASS; }
bool mxIsComplex(const mxArray *a) { return a && a->complex; }
bool mxIsStruct(const mxArray *a) { return a && a->cls == mxSTRUCT_CLASS; }
mxClassID mxGetClassID(const mxArray *a) { return a ? a->cls : mxUNKNOWN_CLASS; }
size_t mxGetNumberOfElements(const mxArray *a) {
  size_t n = 1;
  for (mwSize i = 0; i < a->nd; ++i) n *= a->dims[i];
  return n;
}
bool mxIsEmpty(const mxArray *a) { return mxGetNumberOfElements(a) == 0; }
mwSize mxGetNumberOfDimensions(const mxArray *a) { return a->nd; }
const mwSize *mxGetDimensions(const mxArray *a) { return a->dims; }
size_t mxGetM(const mxArray *a) { return a->dims[0]; }
size_t mxGetN(const mxArray *a) {
  size_t n = 1;
  for (mwSize i = 1; i < a->nd; ++i) n *= a->dims[i];
  return n;
}
void *mxGetData(const mxArray *a) { return a->data; }
double *mxGetDoubles(const mxArray *a) { return (a->cls == mxDOUBLE_CLASS && !a->complex) ? (double *)a->data : NULL; }
mxComplexDouble *mxGetComplexDoubles(const mxArray *a) {
  return (a->cls == mxDOUBLE_CLASS && a->complex) ? (mxComplexDouble *)a->data : NULL;
}
double mxGetScalar(const mxArray *a) {
  if (!a || !a->data || mxIsEmpty(a)) return 0.0;
  switch (a->cls) {
    case mxDOUBLE_CLASS: return *(double *)a->data;
    case mxSINGLE_CLASS: return *(float *)a->data;
    case mxINT8_CLASS: return *(int8_t *)a->data;
    case mxUINT8_CLASS: case mxLOGICAL_CLASS: case mxCHAR_CLASS: return *(uint8_t *)a->data;
    case mxINT16_CLASS: return *(int16_t *)a->data;
    case mxUINT16_CLASS: return *(uint16_t *)a->data;
    case mxINT32_CLASS: return *(int32_t *)a->data;
    case mxUINT32_CLASS: return *(uint32_t *)a->data;
    case mxINT64_CLASS: return (double)*(int64_t *)a->data;
    case mxUINT64_CLASS: return (double)*(uint64_t *)a->data;
    default: return 0.0;
  }
}
int mxGetString(const mxArray *a, char *buf, mwSize len) {
  if (!a || a->cls != mxCHAR_CLASS || len == 0) return 1;
  const size_t n = mxGetNumberOfElements(a);
  const size_t k = n < len - 1 ? n : len - 1;
  memcpy(buf, a->data, k);
  buf[k] = 0;
  return n < len ? 0 : 1;
}
static int field_index(const mxArray *s, const char *name) {
  for (int i = 0; i < s->nfields; ++i)
    if (!strcmp(s->names[i], name)) return i;
  return -1;
}
mxArray *mxGetField(const mxArray *s, mwIndex i, const char *name) {
  if (!s || s->cls != mxSTRUCT_CLASS || i != 0) return NULL;
  const int f = field_index(s, name);
  return f < 0 ? NULL : s->values[f];
}
void mxSetField(mxArray *s, mwIndex i, const char *name, mxArray *v) {
  if (!s || s->cls != mxSTRUCT_CLASS || i != 0) return;
  int f = field_index(s, name);
  if (f < 0) {  /* MATLAB's mxSetField needs an existing field; the shim adds it (test builders) */
    s->names = (char **)realloc(s->names, (size_t)(s->nfields + 2) * sizeof(char *));
    s->values = (mxArray **)realloc(s->values, (size_t)(s->nfields + 2) * sizeof(mxArray *));
    f = s->nfields++;
    s->names[f] = strdup(name);
    s->values[f] = NULL;
  }
  s->values[f] = v;  /* the old value is not freed: MATLAB leaves that to the caller too */
}

/* ---- entry points for tests/mexshim.py ------------------------------------ */
mxArray *shim_numeric(int cls, int nd, const size_t *dims, const void *data, int cplx) {
  mxArray *a = make((mxClassID)cls, cplx, (mwSize)nd, dims);
  if (data && a->data) memcpy(a->data, data, mxGetNumberOfElements(a) * esize(a->cls) * (cplx ? 2 : 1));
  return a;
}
mxArray *shim_string(const char *s) {
  mwSize d[2] = {1, strlen(s)};
  mxArray *a = make(mxCHAR_CLASS, 0, 2, d);
  memcpy(a->data, s, d[1]);
  return a;
}
mxArray *shim_struct(void) { return mxCreateStructMatrix(1, 1, 0, NULL); }
void shim_set_field(mxArray *s, const char *name, mxArray *v) { mxSetField(s, 0, name, v); }
mxArray *shim_get_field(const mxArray *s, const char *name) { return mxGetField(s, 0, name); }
int shim_nfields(const mxArray *s) { return s && s->cls == mxSTRUCT_CLASS ? s->nfields : 0; }
const char *shim_field_name(const mxArray *s, int i) { return s->names[i]; }
/* class, complexity, dims (up to 8) and the payload pointer of an array */
int shim_info(const mxArray *a, int *cls, int *cplx, size_t *dims, void **data) {
  if (!a) return -1;
  *cls = (int)a->cls;
  *cplx = a->complex;
  for (mwSize i = 0; i < a->nd; ++i) dims[i] = a->dims[i];
  *data = a->data;
  return (int)a->nd;
}
void shim_destroy(mxArray *a) { mxDestroyArray(a); }
const char *shim_last_error(void) { return g_msg; }
/* One mexFunction call: 0 = returned, 1 = raised an error (shim_last_error).  After an
 * error the outputs it had created are destroyed and plhs reset to NULL. */
int shim_call(int nlhs, mxArray **plhs, int nrhs, mxArray **prhs) {
  jmp_buf jb;
  g_msg[0] = 0;
  for (int i = 0; i < nlhs; ++i) plhs[i] = NULL;
  if (setjmp(jb)) {
    g_jmp = NULL;
    free_blocks();
    for (int i = 0; i < nlhs; ++i) {
      mxDestroyArray(plhs[i]);
      plhs[i] = NULL;
    }
    return 1;
  }
  g_jmp = &jb;
  mexFunction(nlhs, plhs, nrhs, (const mxArray **)prhs);
  g_jmp = NULL;
  free_blocks();
  return 0;
}

/* mexAtExit: MATLAB runs the registered function at `clear mex` / exit; the shim runs
 * it from shim_clear_mex() (the last registration wins, as in MATLAB). */
static void (*g_atexit)(void);
int mexAtExit(void (*fn)(void)) {
  g_atexit = fn;
  return 0;
}
int shim_clear_mex(void) {
  if (!g_atexit) return 0;
  g_atexit();
  g_atexit = NULL;
  return 1;
}
