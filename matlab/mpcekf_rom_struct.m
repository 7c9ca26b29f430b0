function R = mpcekf_rom_struct(ROM, ntheta, TdegC)
% MPCEKF_ROM_STRUCT  The reference ROM struct (runMPC.m:5) as the plain arrays of the
% library's mpcekf_rom (include/mpcekf.h): what mpcekf_mex('create', R, ...) takes and
% what mpcekf_export_rom writes to JSON.  Defaults: ntheta = 101, TdegC = 6 points from
% 10 degC below the coldest to 10 degC above the warmest ROM set-point.
  if nargin < 2 || isempty(ntheta), ntheta = 101; end
  if nargin < 3 || isempty(TdegC)
    TdegC = linspace(min(ROM.xraData.T) - 10, max(ROM.xraData.T) + 10, 6);
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
  R.F = cd.const.F;  R.R = cd.const.R;  R.Q = fn.const.Q();  R.Rc = fn.const.Rc();  R.Tref = 298.15;
  R.tab_T_K = TK;
  R.neg = mpcekf_tabulate_electrode(fn.neg, th, TK);
  R.pos = mpcekf_tabulate_electrode(fn.pos, th, TK);
end
