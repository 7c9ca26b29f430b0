function [uk, mpcData] = iterMPC(xk, cellState, mpcData)
% Drop-in for iterMPC.m:1 over the MI355X library (mpcekf_mpc_step_ex): the linearisation
% is EKFmatsHandler's device-resident records (cellState.MPC.lin empty) or, when a caller
% built cellState.MPC.lin itself, those 35 x ncells records; their xhat rows are the
% caller's xk (6 x ncells, the state iterMPC.m:29 augments) -- written to the device only
% when xk is not the xhat the device records hold now (the session tracks it: the last
% EKFmatsHandler's xhat, or the xk an earlier iterMPC wrote over it), so a call without an
% override after one with it restores EKFmatsHandler's xhat as the reference would.  uk_1 and the Hildreth warm start live
% in the context.  When runMPC.m has set mpcData.k, row k of mpcData.cost
% (iterMPC.m:89-95: t, J_uncon, J_final, norm_DU, viol, nexec) is filled, one column per
% cell.
  S = mpcekf_session('get');
  lin = cellState.MPC.lin;
  if isempty(lin)
    n = size(cellState.MPC.xhat, 2);
    if isempty(xk), xk = cellState.MPC.xhat; end
    xk = reshape(xk, 6, []) .* ones(1, n);
    if ~isequal(xk, S.xhat_dev)                               % what the device records hold
      mpcekf_mex('linfields', S.h, 30:35, xk);                % MPCEKF_LIN_XHAT
      mpcekf_session('set', 'xhat_dev', xk);
    end
  else
    n = size(lin, 2);
    if ~isempty(xk)
      lin(30:35, :) = reshape(xk, 6, []) .* ones(1, n);      % MPCEKF_LIN_XHAT
    end
  end
  % iterMPC.m:53-60 stability analysis (before the solve: it uses this step's uk_1)
  [mpcData.poles, mpcData.sv] = mpcekf_mex('mpcdiag', S.h, lin, []);
  [uk, nexec, J_unc, J_fin, ndu, nviol] = mpcekf_mex('mpc', S.h, lin, reshape(mpcData.SOCk_1 .* ones(1, n), 1, n));
  mpcData.uk_1 = uk;
  mpcData.nexec = double(nexec);
  if isfield(mpcData, 'cost') && isfield(mpcData, 'k')
    k = mpcData.k;
    if isfield(mpcData, 'Ts'), Ts = mpcData.Ts; else, Ts = cellState.Ts; end
    mpcData.cost.t(k, 1) = (k - 1) * Ts;
    mpcData.cost.J_uncon(k, 1:n) = J_unc;
    mpcData.cost.J_final(k, 1:n) = J_fin;
    mpcData.cost.norm_DU(k, 1:n) = ndu;
    mpcData.cost.viol(k, 1:n) = double(nviol);
    mpcData.cost.nexec(k, 1:n) = double(nexec);
  end
end
