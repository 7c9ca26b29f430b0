function err = mpcekf_check_tables(f, e, Tref, R)
% MPCEKF_CHECK_TABLES  Max abs error of the tabulated electrode model against the
% original cellData.function handles at 1001 interior points and 3 temperatures.
% The MI355X library reproduces the tables bit-for-bit; this number is the part of
% any real-MATLAB parity gap that comes from tabulation rather than the kernels.
  th = linspace(0.001, 0.999, 1001);
  U = e.U.data;  dUdT = e.dUdT.data;  dU = e.dU.data;
  lin = @(tab, x) interp1(linspace(0, 1, numel(tab)), tab, x, 'linear');
  err = struct('Uocp', 0, 'dUocp', 0, 'k0', 0);
  for T = Tref + [-10 0 10]
    Ut = arrayfun(@(t) f.Uocp(t, T), th);
    err.Uocp = max(err.Uocp, max(abs(Ut - (lin(U, th) + (T - Tref) * lin(dUdT, th)))));
    err.dUocp = max(err.dUocp, max(abs(arrayfun(@(t) f.dUocp(t, T), th) - lin(dU, th))));
    k = e.k0ref * exp(e.Ea_k0 / R * (1/Tref - 1/T));
    err.k0 = max(err.k0, abs(f.k0(0.5, T) - k) / abs(f.k0(0.5, T)));
  end
end
