function [uk, mpcData] = iterMPC(xk, cellState, mpcData)
% Drop-in for iterMPC.m:1 over the MI355X library (mpcekf_mpc_step): the state is the
% xhat of cellState.MPC.lin (EKFmatsHandler's, which runMPC.m:101 passes as xk), uk_1
% and the Hildreth warm start live in the context.  mpcData.cost.nexec(k) is filled
% when runMPC.m has set mpcData.k.
  S = mpcekf_session('get');
  lin = cellState.MPC.lin;
  n = size(lin, 2);
  % iterMPC.m:53-60 stability analysis (before the solve: it uses this step's uk_1)
  [mpcData.poles, mpcData.sv] = mpcekf_mex('mpcdiag', S.h, lin, []);
  [uk, nexec] = mpcekf_mex('mpc', S.h, lin, reshape(mpcData.SOCk_1 .* ones(1, n), 1, n));
  mpcData.uk_1 = uk;
  if isfield(mpcData, 'cost') && isfield(mpcData, 'k')
    mpcData.cost.nexec(mpcData.k) = double(nexec(1));
  end
  xk = []; %#ok<NASGU> (the library uses the linearisation record's xhat)
end
