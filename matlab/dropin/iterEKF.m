function [zk,boundzk,ekfData,Xind] = iterEKF(vk,ik,Tk,ekfData)
% Drop-in for UTILITY/iterEKF.m:30 over the MI355X library (mpcekf_ekf_step): zk and
% boundzk are (nz+2) x ncells, Xind.theT / theZ / gamma 4 x ncells (1-based set-point
% indices as the reference's), Xind.model the library's 0-based model index.  zk and Xind
% also stay on the device: Xind.tick names this call, and EKFmatsHandler passes nothing
% back when it gets this call's Xind and zk unchanged (runMPC.m:91 -> :94).
  S = mpcekf_session('get');
  n = numel(vk);
  if any(Tk > 100), Tk = Tk - 273.15; end                    % the library takes degC
  [zk, boundzk, xm, xg] = mpcekf_mex('ekf', S.h, reshape(vk, 1, n), reshape(ik .* ones(1, n), 1, n), ...
                                     reshape(Tk .* ones(1, n), 1, n));
  nZ = numel(ekfData.ROM.xraData.SOC);
  tick = S.ekf_tick + 1;
  mpcekf_session('set', 'ekf_tick', tick);
  mpcekf_session('set', 'zk_last', zk);                      % shared copy (copy-on-write): no data copied
  Xind = struct('gamma', xg, 'theT', double(idivide(xm, int32(nZ))) + 1, 'theZ', double(mod(xm, nZ)) + 1, ...
                'model', xm, 'tick', tick);
  [s, warn, status] = mpcekf_mex('scalars', S.h, [3 4 5]);   % x0, SigmaX0, priorI: 32 B per cell
  ekfData.x0 = s(1, :);  ekfData.SigmaX0 = s(2, :);  ekfData.priorI = s(3, :);
  ekfData.status = status;  ekfData.warnCount = warn;
end
