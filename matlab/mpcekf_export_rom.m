function mpcekf_export_rom(matFile, jsonFile, ntab)
% MPCEKF_EXPORT_ROM  Tabulate a reference ROM (.mat) into the JSON file the MI355X
% framework loads with ROM.load_json (mpc-ekf4fastcharge_amd/rom.py).
%
%   mpcekf_export_rom('ROM_NMC30_HRA.mat', 'rom_nmc30.json')        % 201-point tables
%   mpcekf_export_rom('ROM_NMC30_HRA.mat', 'rom_nmc30.json', 401)
%
% Runs on a machine with MATLAB and the reference's ROM file (runMPC.m:4-5; the file
% is listed in .MISSING_LARGE_BLOBS:1 and is not in this repository).  The
% cellData.function handles are called exactly as the hot path calls them:
%   soc(z,T)       OB_step.m:231-232, iterEKF.m:282-283
%   Uocp(theta,T)  iterEKF.m:362-363, EKFmatsHandler.m:96 (1-arg call -> Tref)
%   dUocp(theta,T) iterEKF.m:392-407, EKFmatsHandler.m:53-92
%   k0(theta,T), Rf(theta,T), wDL(theta,T), Cdl(theta,T), nDL(), theta0(), theta100()
%                  OB_step.m:205-219, 313-314, 329-340
%   const.Q(), const.Rc()                      initMPC.m:66-67, OB_step.m:206
% and tabulated into the library's electrode model (include/mpcekf.h, mpcekf_electrode):
%   U(theta)    = Uocp(theta,Tref)             on ntab uniform points over [0,1]
%   dUdT(theta) = Uocp(theta,Tref+1) - Uocp(theta,Tref)   (per kelvin)
%   dU(theta)   = dUocp(theta,Tref)
%   k0(theta,T) = k0ref*exp(Ea_k0/R*(1/Tref-1/T)), Ea_k0 fitted from Tref and Tref+10
%   Rf, wDL, Cdl at theta = 0.5, T = Tref (the reference uses them as cell constants,
%   OB_step.m:313-314 evaluates wDL/Cdl at SOC0 only)
% The approximation error of the tables is reported by mpcekf_check_tables below.
%
% Every array is written as {"shape": size(X), "order": "F", "data": X(:)'} so the
% loader needs no knowledge of MATLAB's N-D jsonencode nesting.
  if nargin < 3, ntab = 201; end
  S = load(matFile);
  if isfield(S, 'ROM'), ROM = S.ROM; else, f = fieldnames(S); ROM = S.(f{1}); end
  cd = ROM.cellData;  fn = cd.function;  Tref = 298.15;
  th = linspace(0, 1, ntab);

  out = struct();
  out.format = 'mpcekf-rom-v1';
  out.source = matFile;
  out.T_degC = arr(ROM.xraData.T(:)');
  out.SOC_pct = arr(ROM.xraData.SOC(:)');
  out.Ts = ROM.xraData.Tsamp;
  [A, C, D, names, xloc] = mpcekf_pack_models(ROM);
  out.A = arr(A);  out.C = arr(C);  out.D = arr(D);
  out.names = names;                       % cellstr, tfData.names order
  out.xloc = arr(xloc(:)');
  out.F = cd.const.F;  out.R = cd.const.R;
  out.Q = fn.const.Q();  out.Rc = fn.const.Rc();  out.Tref = Tref;
  out.neg = electrode(fn.neg, th, Tref, cd.const.R);
  out.pos = electrode(fn.pos, th, Tref, cd.const.R);
  out.tab_error = struct('neg', mpcekf_check_tables(fn.neg, out.neg, Tref, cd.const.R), ...
                         'pos', mpcekf_check_tables(fn.pos, out.pos, Tref, cd.const.R));

  fid = fopen(jsonFile, 'w');
  assert(fid > 0, 'mpcekf_export_rom: cannot open %s', jsonFile);
  fprintf(fid, '%s', jsonencode(out));
  fclose(fid);
end

function e = electrode(f, th, Tref, R)
  e = struct();
  e.theta0 = f.theta0();  e.theta100 = f.theta100();
  e.Rf = f.Rf(0.5, Tref);
  e.k0ref = f.k0(0.5, Tref);
  e.Ea_k0 = R * log(f.k0(0.5, Tref + 10) / e.k0ref) / (1/Tref - 1/(Tref + 10));
  e.wDL = f.wDL(0.5, Tref);  e.Cdl = f.Cdl(0.5, Tref);  e.nDL = f.nDL();
  U = arrayfun(@(t) f.Uocp(t, Tref), th);
  e.U = arr(U);
  e.dUdT = arr(arrayfun(@(t) f.Uocp(t, Tref + 1), th) - U);
  e.dU = arr(arrayfun(@(t) f.dUocp(t, Tref), th));
end

function a = arr(X)
  a = struct('shape', size(X), 'order', 'F', 'data', reshape(double(X), 1, []));
end
