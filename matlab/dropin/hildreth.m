function [DU, lambda, nexec] = hildreth(E, F, M, gamma, lambda0, maxIter)
% Drop-in for hildreth.m:1 over the MI355X library (mpcekf_hildreth, one problem).
  [DU, lambda, nexec] = mpcekf_mex('hildreth', E, F(:), M, gamma(:), lambda0(:), maxIter);
end
