function kfData = initKF(SOC0,T0,SigmaX0,SigmaV,SigmaW,blend,ROMs)
% Drop-in for UTILITY/initKF.m:30 over the MI355X library (include/mpcekf.h).  Put
% matlab/dropin ahead of the reference on the path; runMPC.m then runs unchanged.
% The settings are recorded; the library context (initKF + initMPC + the plant's first
% call, mpcekf_init_cells) is created on the first OB_step call, which brings SOC0/Tc.
% SOC0 and T0 may be vectors: one cell each (the batch).
  if any(T0 > 100), T0 = T0 - 273.15; end                    % initKF.m:38-41: K -> degC
  m = upper(blend);
  if any(strcmp(m, {'OB', 'OUTB'})), m = 'OB';
  elseif any(strcmp(m, {'MB', 'MDLB'})), m = 'MB';
  else, error('Unknown blend method (initKF.m:44-49)'); end
  kfData = struct('SOC', SOC0/100, 'SOC0', SOC0/100, 'T', T0 + 273.15, 'SigmaX0', diag(SigmaX0)', ...
                  'SigmaV', SigmaV, 'SigmaW', SigmaW, 'method', m, 'ROM', ROMs, ...
                  'nz', numel(ROMs.tfData.names), 'xhat', zeros(size(ROMs.ROMmdls(1,1).A, 1), 1), ...
                  'Ts', ROMs.xraData.Tsamp, 'Q', ROMs.cellData.function.const.Q());
  mpcekf_session('reset');
  mpcekf_session('set', 'kf', kfData);
end
