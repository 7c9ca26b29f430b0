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
    % Tc of thousands of distinct values), built as mpcekf_export_rom builds them
    % (mpcekf_build_tables: node tables for lookup-table handles, ntheta by the error
    % budget) with the budget checked at the distinct Tc this run uses.  A ROM whose tables
    % miss the budget there is refused ('mpcekf:budget'), unless initCfg.tabBudget = 'warn':
    % then it runs with a warning and cellState.tab_error says how far its lookups are off.
    Tu = unique(Tc(:)');
    [R, terr, tok] = mpcekf_build_tables(ROM, [], Tu, struct('Teval', Tu + 273.15, 'strict', false));
    if ~tok
      msg = sprintf(['OB_step drop-in: the electrode tables miss the error budget at the run''s ' ...
                     'temperatures (neg Uocp %.3g V, k0 %.3g; pos Uocp %.3g V, k0 %.3g)'], ...
                    terr.neg.Uocp, terr.neg.k0_rel, terr.pos.Uocp, terr.pos.k0_rel);
      if isfield(initCfg, 'tabBudget') && strcmpi(initCfg.tabBudget, 'warn')
        warning('mpcekf:budget', '%s', msg);
      else
        error('mpcekf:budget', '%s (initCfg.tabBudget = ''warn'' runs it anyway)', msg);
      end
    end
    h = mpcekf_mex('create', R, cfg, S.device, n);
    mpcekf_session('set', 'h', h);
    mpcekf_mex('init', h, reshape(initCfg.SOC0, 1, n), Tc .* ones(1, n));
    fn = ROM.cellData.function.neg;
    cellState = struct('initialized', true, 'h', h, 'n', n, 'Ts', ROM.xraData.Tsamp, ...
                       'theta0n', fn.theta0(), 'theta100n', fn.theta100(), 'tab_error', terr);
  end
  n = cellState.n;
  s = mpcekf_mex('scalars', cellState.h, [1 2]);             % pre-update averages (OB_step.m:226-228),
  obs = struct('negSOC', s(1, :), 'posSOC', s(2, :));         % 16 B per cell over PCIe
  obs.cellSOC = (obs.negSOC - cellState.theta0n) / (cellState.theta100n - cellState.theta0n);
  Vcell = mpcekf_mex('plant', cellState.h, reshape(Iapp .* ones(1, n), 1, n), reshape(Tc .* ones(1, n), 1, n));
  obs.Vcell = Vcell;
end
