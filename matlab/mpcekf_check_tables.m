function err = mpcekf_check_tables(f, e, th, TK)
% MPCEKF_CHECK_TABLES  Max abs error of the library's bilinear (theta, T) tables against
% the original cellData.function handles, at 997 interior theta points and at every
% table temperature and the midpoints between them, plus the deviation of soc(z,T) from
% the linear-in-z form the library assumes.  The library reproduces the tables
% bit-for-bit; this is the tabulation part of any real-MATLAB parity gap.
  x = linspace(0.001, 0.999, 997);
  Ts = sort([TK, (TK(1:end-1) + TK(2:end)) / 2]);
  tab = @(t2, xx, T) bilin(reshape(t2.data, t2.shape), th, TK, xx, T);
  err = struct('Uocp', 0, 'dUocp', 0, 'k0_rel', 0, 'Rf_rel', 0, 'Cdleff_rel', 0, 'soc_lin', 0);
  nDL = f.nDL();
  for T = Ts
    err.Uocp = max(err.Uocp, max(abs(arrayfun(@(t) f.Uocp(t, T), x) - tab(e.Uocp, x, T))));
    err.dUocp = max(err.dUocp, max(abs(arrayfun(@(t) f.dUocp(t, T), x) - tab(e.dUocp, x, T))));
    k = arrayfun(@(t) f.k0(t, T), x);
    err.k0_rel = max(err.k0_rel, max(abs(k - tab(e.k0, x, T)) ./ abs(k)));
    r = arrayfun(@(t) f.Rf(t, T), x);
    err.Rf_rel = max(err.Rf_rel, max(abs(r - tab(e.Rf, x, T)) ./ max(abs(r), eps)));
    c = arrayfun(@(t) f.Cdl(t, T)^(2 - nDL) * f.wDL(t, T)^(nDL - 1), x);
    err.Cdleff_rel = max(err.Cdleff_rel, max(abs(c - tab(e.Cdleff, x, T)) ./ abs(c)));
    s0 = f.soc(0, T);  s1 = f.soc(1, T);
    err.soc_lin = max(err.soc_lin, max(abs(arrayfun(@(z) f.soc(z, T), x) - (s0 + x * (s1 - s0)))));
  end
end

function v = bilin(t2, th, TK, x, T)
  % the library's evaluation order (include/mpcekf.h): theta rows first, then T
  rows = interp1(th, t2.', min(max(x, 0), 1), 'linear').';   % [ntemp, numel(x)]
  if numel(TK) == 1, v = rows; return; end
  Tc = min(max(T, TK(1)), TK(end));
  j = find(TK <= Tc, 1, 'last');  j = min(j, numel(TK) - 1);
  g = (Tc - TK(j)) / (TK(j + 1) - TK(j));
  v = rows(j, :) + g * (rows(j + 1, :) - rows(j, :));
end
