function [MPC, xhat] = EKFmatsHandler(ekfData, Xind, zk, Tk)
% Drop-in for EKFmatsHandler.m:1 over the MI355X library (mpcekf_linearize).  MPC holds
% the first cell's matrices in the reference's shapes plus MPC.lin, the 35 x ncells
% linearisation records (include/mpcekf.h MPCEKF_LIN_*) iterMPC hands back to the
% library; xhat is 6 x ncells.
  S = mpcekf_session('get');
  n = size(zk, 2);
  lin = mpcekf_mex('linearize', S.h, zk, Xind.model, Xind.gamma, reshape(Tk .* ones(1, n), 1, n));
  MPC = struct('A', diag(lin(1:6, 1)), 'B', ones(6, 1), 'Csoc', lin(7:12, 1)', 'Dsoc', lin(13, 1), ...
               'Cv', lin(14:19, 1)', 'Dv', lin(20, 1), 'Cphi', lin(21:26, 1)', 'Dphi', lin(27, 1), ...
               'bv', lin(28, 1), 'bphi', lin(29, 1), 'lin', lin);
  [~, imax] = max(Xind.gamma(:, 1));
  MPC.iT = Xind.theT(imax, 1);  MPC.iZ = Xind.theZ(imax, 1);  MPC.pickWeight = Xind.gamma(imax, 1);
  xhat = lin(30:35, :);
end
