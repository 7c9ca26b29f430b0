function S = mpcekf_session(op, name, value)
% MPCEKF_SESSION  State the drop-in wrappers share within one MATLAB session: the
% library context handle (one context for the batch, like the reference's one
% persistent iterEKF state per session, iterEKF.m:31) and the initKF / initMPC settings
% the context is created from on the first OB_step call.
%   S = mpcekf_session('get');  mpcekf_session('set', name, value);  mpcekf_session('reset')
  persistent P
  % zk_last / ekf_tick: the zk the last iterEKF returned and a counter of iterEKF calls, so
  % EKFmatsHandler knows when the library's device copies of zk and Xind are the caller's
  % xhat_dev: the xhat the device-resident linearisation records hold (EKFmatsHandler's, or
  % the xk an iterMPC call wrote over it)
  if isempty(P), P = struct('h', [], 'kf', [], 'mpc', [], 'device', 0, 'zk_last', [], 'ekf_tick', 0, ...
                            'xhat_dev', []); end
  switch op
    case 'set'
      P.(name) = value;
    case 'reset'
      if ~isempty(P.h), mpcekf_mex('destroy', P.h); end
      P.h = [];
    case 'get'
    otherwise
      error('mpcekf_session: unknown op %s', op);
  end
  S = P;
end
