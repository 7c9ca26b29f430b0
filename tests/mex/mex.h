/*
 * mex.h -- test shim of the MATLAB MEX API (R2018a interleaved-complex subset).
 *
 * NOT MATLAB.  Just enough of the documented MEX/mx* interface for
 * matlab/mpcekf_mex.c to compile and run without MATLAB, so the gateway's
 * column-major marshalling can be driven from tests/test_mex_gateway.py and
 * compared with the ctypes path.  Implementation: tests/mex/mexshim.c.
 */
#ifndef MPCEKF_TEST_MEX_H
#define MPCEKF_TEST_MEX_H
#include "matrix.h"

#ifdef __cplusplus
extern "C" {
#endif

void mexErrMsgIdAndTxt(const char *id, const char *fmt, ...) __attribute__((noreturn));
void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[]);
int mexAtExit(void (*fn)(void));

#ifdef __cplusplus
}
#endif
#endif
