function e = mpcekf_tabulate_electrode(f, th, TK)
% MPCEKF_TABULATE_ELECTRODE  One electrode's cellData.function handles on the (T, theta)
% grid TK (K, 1..8 ascending) x th (uniform over [0, 1]): the fields of the library's
% mpcekf_electrode (include/mpcekf.h), 2-D tables as ntemp x ntheta.  The handles are
% called as the hot path calls them (see mpcekf_export_rom for the file:line list).
  nt = numel(TK);  nth = numel(th);
  e = struct();
  e.theta0 = f.theta0();  e.theta100 = f.theta100();
  e.soc0 = arrayfun(@(T) f.soc(0, T), TK);
  e.soc100 = arrayfun(@(T) f.soc(1, T), TK);
  [U, dU, K0, RF, CDL] = deal(zeros(nt, nth));
  nDL = f.nDL();
  for j = 1:nt
    T = TK(j);
    U(j, :) = arrayfun(@(t) f.Uocp(t, T), th);
    dU(j, :) = arrayfun(@(t) f.dUocp(t, T), th);
    K0(j, :) = arrayfun(@(t) f.k0(t, T), th);
    RF(j, :) = arrayfun(@(t) f.Rf(t, T), th);
    CDL(j, :) = arrayfun(@(t) f.Cdl(t, T)^(2 - nDL) * f.wDL(t, T)^(nDL - 1), th);   % OB_step.m:212-219
  end
  e.Uocp = U;  e.dUocp = dU;  e.k0 = K0;  e.Rf = RF;  e.Cdleff = CDL;
  try
    e.Uocp1 = arrayfun(@(t) f.Uocp(t), th);          % EKFmatsHandler.m:96, one argument
  catch
    e.Uocp1 = arrayfun(@(t) f.Uocp(t, 298.15), th);  % a handle that needs T: Tref
  end
end
