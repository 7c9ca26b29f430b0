function [Vcell, obs, cellState] = OB_step(Iapp, Tc, cellState, ROM, initCfg)
% Drop-in for OB_step.m:1 over the MI355X library: the first call (empty cellState)
% creates the context from ROM and the recorded initKF / initMPC settings and runs
% mpcekf_init_cells; every call then runs the plant step (mpcekf_plant_step) at Tc for
% all cells.  cellState carries the handle; obs holds Vcell only (the library returns
% the voltage; the other observables stay on the device).
  if nargin < 3 || isempty(cellState) || ~isfield(cellState, 'initialized') || ~cellState.initialized
    if nargin < 5 || ~isfield(initCfg, 'SOC0')
      error('First call requires initCfg.SOC0 (in %).');
    end
    S = mpcekf_session('get');
    if isempty(S.kf) || isempty(S.mpc), error('mpcekf drop-in: call initKF and initMPC first'); end
    n = numel(initCfg.SOC0);
    cfg = S.mpc.mpcekf_cfg;
    cfg.SigmaV = S.kf.SigmaV;  cfg.SigmaW = S.kf.SigmaW;  cfg.SigmaX0 = S.kf.SigmaX0;
    cfg.flags = int32(1);                                  % MPCEKF_CF_BOUNDS: boundzk too
    if strcmp(S.kf.method, 'MB'), cfg.method = 1; end
    h = mpcekf_mex('create', mpcekf_rom_struct(ROM), cfg, S.device, n);
    mpcekf_session('set', 'h', h);
    mpcekf_mex('init', h, reshape(initCfg.SOC0, 1, n), Tc .* ones(1, n));
    cellState = struct('initialized', true, 'h', h, 'n', n, 'Ts', ROM.xraData.Tsamp);
  end
  n = cellState.n;
  Vcell = mpcekf_mex('plant', cellState.h, reshape(Iapp .* ones(1, n), 1, n), reshape(Tc .* ones(1, n), 1, n));
  obs = struct('Vcell', Vcell);
end
