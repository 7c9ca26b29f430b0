/*
 * matrix.h -- test shim of MATLAB's mx* array API (see mex.h; NOT MATLAB).
 * Arrays are column-major with MATLAB's class ids; complex doubles are
 * interleaved (re, im) as in the R2018a API.
 */
#ifndef MPCEKF_TEST_MATRIX_H
#define MPCEKF_TEST_MATRIX_H
#include <stdbool.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef size_t mwSize;
typedef size_t mwIndex;
typedef struct mxArray_tag mxArray;
typedef enum {
  mxUNKNOWN_CLASS = 0, mxCELL_CLASS, mxSTRUCT_CLASS, mxLOGICAL_CLASS, mxCHAR_CLASS, mxVOID_CLASS,
  mxDOUBLE_CLASS, mxSINGLE_CLASS, mxINT8_CLASS, mxUINT8_CLASS, mxINT16_CLASS, mxUINT16_CLASS,
  mxINT32_CLASS, mxUINT32_CLASS, mxINT64_CLASS, mxUINT64_CLASS
} mxClassID;
typedef enum { mxREAL = 0, mxCOMPLEX = 1 } mxComplexity;
typedef struct {
  double real, imag;
} mxComplexDouble;

void *mxMalloc(size_t n);
void mxFree(void *p);
mxArray *mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity c);
mxArray *mxCreateDoubleScalar(double v);
mxArray *mxCreateNumericMatrix(mwSize m, mwSize n, mxClassID cls, mxComplexity c);
mxArray *mxCreateStructMatrix(mwSize m, mwSize n, int nfields, const char **names);
void mxDestroyArray(mxArray *a);
bool mxIsDouble(const mxArray *a);
bool mxIsInt32(const mxArray *a);
bool mxIsUint64(const mxArray *a);
bool mxIsNumeric(const mxArray *a);
bool mxIsComplex(const mxArray *a);
bool mxIsStruct(const mxArray *a);
bool mxIsEmpty(const mxArray *a);
mxClassID mxGetClassID(const mxArray *a);
size_t mxGetNumberOfElements(const mxArray *a);
mwSize mxGetNumberOfDimensions(const mxArray *a);
const mwSize *mxGetDimensions(const mxArray *a);
size_t mxGetM(const mxArray *a);
size_t mxGetN(const mxArray *a);
void *mxGetData(const mxArray *a);
double *mxGetDoubles(const mxArray *a);
mxComplexDouble *mxGetComplexDoubles(const mxArray *a);
double mxGetScalar(const mxArray *a);
int mxGetString(const mxArray *a, char *buf, mwSize len);
mxArray *mxGetField(const mxArray *s, mwIndex i, const char *name);
void mxSetField(mxArray *s, mwIndex i, const char *name, mxArray *v);

#ifdef __cplusplus
}
#endif
#endif
