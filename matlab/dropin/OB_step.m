function [Vcell, obs, cellState] = OB_step(Iapp, Tc, cellState, ROM, initCfg)
% Drop-in for OB_step.m:1 over the MI355X library: the first call (empty cellState)
% creates the context from ROM and the recorded initKF / initMPC settings and runs
% mpcekf_init_cells; every call then runs the plant step (mpcekf_plant_step) at Tc for
% all cells.  cellState carries the handle.  obs holds Vcell and the pre-step
% electrode averages of OB_step.m:226-228 (negSOC, posSOC, cellSOC); the other
% observables of OB_step.m:289-356 stay on the device (runMPC.m reads none of them).
  if nargin < 3 || isempty(cellState) || ~isfield(cellState, 'initialized') || ~cellState.initialized
    if nargin < 5 || ~isfield(initCfg, 'SOC0')
      error('First call requires initCfg.SOC0 (in %).');
    end
    S = mpcekf_session('get');
    if isempty(S.kf) || isempty(S.mpc), error('mpcekf drop-in: call initKF and initMPC first'); end
    n = numel(initCfg.SOC0);
    cfg = S.mpc.mpcekf_cfg;
    cfg.SigmaV = S.kf.SigmaV;  cfg.SigmaW = S.kf.SigmaW;  cfg.SigmaX0 = S.kf.SigmaX0;
    cfg.flags = 1;                                         % MPCEKF_CF_BOUNDS: boundzk too
    if strcmp(S.kf.method, 'MB'), cfg.method = 1; end
    % the electrode tables hold the ROM set-points and the distinct Tc (mpcekf_rom_struct
    % keeps only their span when they do not fit its 8 table temperatures, e.g. a per-cell
    % Tc of thousands of distinct values)
    h = mpcekf_mex('create', mpcekf_rom_struct(ROM, [], [], unique(Tc(:)')), cfg, S.device, n);
    mpcekf_session('set', 'h', h);
    mpcekf_mex('init', h, reshape(initCfg.SOC0, 1, n), Tc .* ones(1, n));
    fn = ROM.cellData.function.neg;
    cellState = struct('initialized', true, 'h', h, 'n', n, 'Ts', ROM.xraData.Tsamp, ...
                       'theta0n', fn.theta0(), 'theta100n', fn.theta100());
  end
  n = cellState.n;
  s = mpcekf_mex('scalars', cellState.h, [1 2]);             % pre-update averages (OB_step.m:226-228),
  obs = struct('negSOC', s(1, :), 'posSOC', s(2, :));         % 16 B per cell over PCIe
  obs.cellSOC = (obs.negSOC - cellState.theta0n) / (cellState.theta100n - cellState.theta0n);
  Vcell = mpcekf_mex('plant', cellState.h, reshape(Iapp .* ones(1, n), 1, n), reshape(Tc .* ones(1, n), 1, n));
  obs.Vcell = Vcell;
end
