function mpcekf_export_rom(matFile, jsonFile, ntheta, TdegC, order)
% MPCEKF_EXPORT_ROM  Tabulate a reference ROM (.mat) into the JSON file the MI355X
% framework loads with ROM.load_json (mpc-ekf4fastcharge_amd/rom.py, format v3 -- v4 when
% a handle is a lookup table on its own breakpoints (node tables, mpcekf_build_tables);
% v2 with order = 1).
%
%   mpcekf_export_rom('ROM_NMC30_HRA.mat', 'rom_nmc30.json')          % quintics, ntheta by budget
%   mpcekf_export_rom('ROM_NMC30_HRA.mat', 'rom_nmc30.json', 1025, [15 25 35])
%   mpcekf_export_rom('ROM_NMC30_HRA.mat', 'rom_nmc30_v2.json', 101, [], 1)   % v2 linear
%
% ABI v3 (order 5, the default; include/mpcekf.h tab_npoly): every row is also a
% piecewise Hermite quintic in theta fitted to the handle's values and derivatives, and a
% handle of Arrhenius form gets its exact factor (mpcekf_tabulate_electrode).  Without an
% explicit ntheta the exporter starts at 257 theta points and doubles them until
% mpcekf_check_tables' budget holds (a tenth of north_star's 1e-6 on phise and V); it
% refuses to write a file whose tables miss the budget at 4097 points.
%
% Runs on a machine with MATLAB and the reference's ROM file (runMPC.m:4-5; the file
% is listed in .MISSING_LARGE_BLOBS:1 and is not in this repository).  Every
% cellData.function handle the hot path calls is evaluated on a (T, theta) grid --
% TdegC (default: 6 points from 10 degC below the coldest to 10 degC above the warmest
% ROM set-point) x ntheta uniform points over [0, 1] -- and written as the library's
% [ntemp][ntheta] tables (include/mpcekf.h, mpcekf_electrode):
%   Uocp(theta,T)   OB_step.m:313-314,337-338; iterEKF.m:362-363,404-405; EKFmatsHandler.m:84-85
%   Uocp(theta)     the one-argument call of EKFmatsHandler.m:96 (its own 1-D table)
%   dUocp(theta,T)  OB_step.m:231-232; iterEKF.m:495-496,579-580
%   k0(theta,T)     OB_step.m:329-330; iterEKF.m:392-393,463-464; EKFmatsHandler.m:60-61
%   Rf(theta,T)     OB_step.m:339-340; iterEKF.m:406-407,441-442; EKFmatsHandler.m:68-69
%   Cdleff(theta,T) = Cdl(theta,T)^(2-nDL) * wDL(theta,T)^(nDL-1)   OB_step.m:212-219
%   soc(0,T), soc(1,T)   soc(z,T) is taken as linear in z (checked)  iterEKF.m:282-283
%   theta0(), theta100(), const.Q(), const.Rc()     OB_step.m:205-210, initMPC.m:66-67
% The library evaluates the tables with a defined bilinear interpolation (theta, then
% T; both clamped to the grid).  mpcekf_check_tables reports how far that is from the
% handles between the grid points: the part of a real-MATLAB parity gap that comes from
% tabulation rather than the kernels.  LDS budget (v2 only): the kernels stage 4
% (plant: 5) of the tables per electrode next to the ROM models, so ntheta x ntemp is
% bounded (mpcekf_ctx_create fails with MPCEKF_E_UNSUPPORTED when they do not fit
% 160 KiB); the v3 polynomials are read from a global (L2-resident) table of any size.
%
% Every array is written as {"shape": size(X), "order": "F", "data": X(:)'} so the
% loader needs no knowledge of MATLAB's N-D jsonencode nesting.
  if nargin < 3, ntheta = []; end
  if nargin < 4, TdegC = []; end
  if nargin < 5 || isempty(order), order = 5; end
  S = load(matFile);
  if isfield(S, 'ROM'), ROM = S.ROM; else, f = fieldnames(S); ROM = S.(f{1}); end
  fn = ROM.cellData.function;
  if order > 1
    % the table step shared with the OB_step drop-in: node tables for lookup-table handles
    % (ABI v4), uniform quintics otherwise, ntheta by the error budget (or the given one,
    % still checked); refuses a file that misses the budget
    R = mpcekf_build_tables(ROM, TdegC, [], struct('order', order, 'ntheta', ntheta));
  else
    R = mpcekf_rom_struct(ROM, ntheta, TdegC, [], order);
  end
  th = linspace(0, 1, size(R.neg.Uocp, 2));

  out = struct();
  out.format = 'mpcekf-rom-v2';
  if order > 1, out.format = 'mpcekf-rom-v3'; end
  if isfield(R.neg, 'nodes') || isfield(R.pos, 'nodes'), out.format = 'mpcekf-rom-v4'; end
  out.source = matFile;
  out.T_degC = arr(R.T_degC);
  out.SOC_pct = arr(R.SOC_pct);
  out.Ts = R.Ts;
  out.A = arr(R.A);  out.C = arr(R.C);  out.D = arr(R.D);
  out.names = R.names;                     % cellstr, tfData.names order
  out.xloc = arr(R.xloc);
  out.F = R.F;  out.R = R.R;  out.Q = R.Q;  out.Rc = R.Rc;  out.Tref = R.Tref;
  out.tab_T_K = arr(R.tab_T_K);
  out.neg = jsonify(R.neg);
  out.pos = jsonify(R.pos);
  out.tab_error = struct('neg', mpcekf_check_tables(fn.neg, R.neg, th, R.tab_T_K, R.Tref, R.R), ...
                         'pos', mpcekf_check_tables(fn.pos, R.pos, th, R.tab_T_K, R.Tref, R.R));

  fid = fopen(jsonFile, 'w');
  assert(fid > 0, 'mpcekf_export_rom: cannot open %s', jsonFile);
  fprintf(fid, '%s', jsonencode(out));
  fclose(fid);
end

function e = jsonify(t)
  e = struct();
  e.theta0 = t.theta0;  e.theta100 = t.theta100;
  e.soc0 = arr(t.soc0);  e.soc100 = arr(t.soc100);
  e.Uocp = arr(t.Uocp);  e.dUocp = arr(t.dUocp);  e.k0 = arr(t.k0);  e.Rf = arr(t.Rf);
  e.Cdleff = arr(t.Cdleff);  e.Uocp1 = arr(t.Uocp1);
  if isfield(t, 'poly')   % v3: {"poly": {"Uocp": {shape, order, data}, ...}, "Ea": {"k0": J/mol, ...}}
    e.poly = struct();
    for k = fieldnames(t.poly)'
      e.poly.(k{1}) = arr(t.poly.(k{1}));
    end
    names = {'Uocp', 'dUocp', 'k0', 'Rf', 'Cdleff'};
    e.Ea = struct();
    for k = 1:5
      if t.Ea(k) ~= 0, e.Ea.(names{k}) = t.Ea(k); end
    end
  end
  if isfield(t, 'nodes')  % v4: {"nodes": {"Uocp": {"x": {shape, order, data}, "p": {...}}, ...}}
    e.nodes = struct();
    for k = fieldnames(t.nodes)'
      e.nodes.(k{1}) = struct('x', arr(t.nodes.(k{1}).x), 'p', arr(t.nodes.(k{1}).p));
    end
  end
end

function a = arr(X)
  a = struct('shape', size(X), 'order', 'F', 'data', reshape(double(X), 1, []));
end
