function [MPC, xhat] = EKFmatsHandler(ekfData, Xind, zk, Tk)
% Drop-in for EKFmatsHandler.m:1 over the MI355X library (mpcekf_linearize).  The 35 x
% ncells linearisation records (include/mpcekf.h MPCEKF_LIN_*) stay on the device for
% iterMPC (MPC.lin = [], MPC.tick names them); MPC carries what runMPC.m:95-96 reads,
% Cphi / Dphi / bphi (one row / value per cell), and xhat is 6 x ncells: 14 doubles per
% cell cross PCIe (mpcekf_lin_fields).  When Xind or zk are not the last iterEKF's as it
% returned them, they are passed to the library (the reference's semantics either way).
  S = mpcekf_session('get');
  n = size(zk, 2);
  tk = reshape(Tk .* ones(1, n), 1, n);
  if isfield(Xind, 'tick') && Xind.tick == S.ekf_tick && isequal(zk, S.zk_last)
    mpcekf_mex('linearize', S.h, [], [], [], tk);            % the device copies of zk and Xind
  else
    mpcekf_mex('linearize', S.h, zk, Xind.model, Xind.gamma, tk);
  end
  f = mpcekf_mex('linfields', S.h, [21:27, 29, 30:35]);      % Cphi (6), Dphi, bphi, xhat (6)
  tick = [];
  if isfield(Xind, 'tick'), tick = Xind.tick; end
  MPC = struct('Cphi', f(1:6, :)', 'Dphi', f(7, :), 'bphi', f(8, :), 'lin', [], 'tick', tick);
  [~, imax] = max(Xind.gamma(:, 1));
  MPC.iT = Xind.theT(imax, 1);  MPC.iZ = Xind.theZ(imax, 1);  MPC.pickWeight = Xind.gamma(imax, 1);
  xhat = f(9:14, :);
  MPC.xhat = xhat;
  mpcekf_session('set', 'xhat_dev', xhat);                   % the device records' xhat (iterMPC)
end
