function [Phi, G, aug] = predMat(A, B, C, D, Np, Nc)
% Drop-in for predMat.m:1 over the MI355X library (mpcekf_predmat): A must be diagonal
% and B all ones, as EKFmatsHandler.m:35-38 builds them (the library's model form).
  assert(isequal(diag(diag(A)), A) && all(B(:) == 1), 'predMat drop-in: diagonal A and unit B only');
  [Phi, G] = mpcekf_mex('predmat', diag(A)', C(:)', D, Np, Nc);
  nx = size(A, 1);                                  % x_aug = [x; u], du input (predMat.m:18-24)
  aug = struct('A', [A, B; zeros(1, nx), 1], 'B', [zeros(nx, 1); 1], 'C', [C, D], 'nx_aug', nx + 1, 'm', 1, 'q', 1);
end
