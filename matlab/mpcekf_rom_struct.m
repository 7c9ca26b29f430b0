function R = mpcekf_rom_struct(ROM, ntheta, TdegC, TC, order, nodes)
% MPCEKF_ROM_STRUCT  The reference ROM struct (runMPC.m:5) as the plain arrays of the
% library's mpcekf_rom (include/mpcekf.h): what mpcekf_mex('create', R, ...) takes and
% what mpcekf_export_rom writes to JSON.
% The electrode functions (k0, Rf, Cdleff, Uocp, dUocp) are tabulated on TdegC and
% interpolated linearly in T between table temperatures; at a table temperature the
% lookup is the handle's value exactly.  Default TdegC: the ROM set-point temperatures,
% the simulation temperatures TC (default 25 degC, runMPC.m:8) and guard points 10 degC
% beyond the coldest / warmest (T is clamped to the table range); spare slots up to 8
% split the widest intervals.
% order (ABI v3, default 5): the rows are also fitted by Hermite quintics (3: cubics) in
% theta and Arrhenius handles get their exact factor (mpcekf_tabulate_electrode): an OCP
% U0(th) + (T - Tref) dU/dT(th) is then exact between table temperatures and k0 / Rf at
% any T; default ntheta 513 (mpcekf_export_rom raises it until mpcekf_check_tables'
% budget holds).  order 1: the v2 linear tables (default ntheta 101), where an Arrhenius
% k0 interpolated linearly in T is off by about h^2/8 (Ea/(R T^2))^2 between table
% points (DESIGN.md 3: ~1.4 % at h = 5 K, Ea = 50 kJ/mol).
% nodes (ABI v4, default false): also the node tables of lookup-table handles
% (mpcekf_tabulate_electrode); mpcekf_build_tables sets it and checks the budget.
% Tref (the Arrhenius reference temperature of the v3 factor) is ROM.cellData.const.Tref
% when the ROM has one, else 298.15 K.
  if nargin < 5 || isempty(order), order = 5; end
  if nargin < 6 || isempty(nodes), nodes = false; end
  if nargin < 2 || isempty(ntheta), ntheta = 101 + 412 * (order > 1); end
  if nargin < 4 || isempty(TC), TC = 25; end
  if nargin < 3 || isempty(TdegC)
    Ts = ROM.xraData.T(:)';
    TCu = unique(TC(:)');
    % more distinct simulation temperatures than free table slots (e.g. a per-cell Tc):
    % keep only their span, the interior is filled by the interval halving below
    if numel(unique([Ts, TCu])) > 8, TCu = unique([min(TCu), max(TCu)]); end
    TdegC = unique([Ts, TCu]);
    if numel(TdegC) > 8                     % set-points + span still too many: the span
      TdegC = linspace(min(TdegC), max(TdegC), 8);  % evenly (lookups off the points interpolate)
    end
    guard = [min(TdegC) - 10, max(TdegC) + 10];
    if numel(TdegC) + 2 <= 8, TdegC = unique([guard(1), TdegC, guard(2)]); end
    while numel(TdegC) < 8                  % spare slots halve the widest intervals
      [~, k] = max(diff(TdegC));
      TdegC = [TdegC(1:k), (TdegC(k) + TdegC(k + 1)) / 2, TdegC(k + 1:end)];
    end
  end
  assert(numel(TdegC) >= 1 && numel(TdegC) <= 8 && all(diff(TdegC) > 0), ...
         'mpcekf_rom_struct: 1..8 ascending table temperatures');
  cd = ROM.cellData;  fn = cd.function;
  TK = TdegC(:)' + 273.15;
  th = linspace(0, 1, ntheta);
  [A, C, D, names, xloc] = mpcekf_pack_models(ROM);
  codes = {'negIfdl','posIfdl','negIf','posIf','negIdl','posIdl','negPhis','posPhis','negPhise', ...
           'posPhise','negThetass','posThetass','negPhie','sepPhie','posPhie','negThetae','sepThetae', ...
           'posThetae'};                                  % MPCEKF_TF_* order
  [ok, code] = ismember(names, codes);
  assert(all(ok), 'mpcekf_rom_struct: unknown tfData.names entry');
  R = struct();
  R.T_degC = ROM.xraData.T(:)';  R.SOC_pct = ROM.xraData.SOC(:)';  R.Ts = ROM.xraData.Tsamp;
  R.A = A;  R.C = C;  R.D = D;
  R.names = names;  R.tf_code = int32(code - 1);  R.xloc = xloc(:)';
  R.F = cd.const.F;  R.R = cd.const.R;  R.Q = fn.const.Q();  R.Rc = fn.const.Rc();
  R.Tref = 298.15;
  if isfield(cd.const, 'Tref') && ~isempty(cd.const.Tref), R.Tref = cd.const.Tref; end
  R.tab_T_K = TK;
  R.neg = mpcekf_tabulate_electrode(fn.neg, th, TK, order, R.Tref, R.R, nodes && order > 1);
  R.pos = mpcekf_tabulate_electrode(fn.pos, th, TK, order, R.Tref, R.R, nodes && order > 1);
end
