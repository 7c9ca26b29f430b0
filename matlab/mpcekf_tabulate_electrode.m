function e = mpcekf_tabulate_electrode(f, th, TK, order, Tref, R, nodes)
% MPCEKF_TABULATE_ELECTRODE  One electrode's cellData.function handles on the (T, theta)
% grid TK (K, 1..8 ascending) x th (uniform over [0, 1]): the fields of the library's
% mpcekf_electrode (include/mpcekf.h), 2-D tables as ntemp x ntheta.  The handles are
% called as the hot path calls them (see mpcekf_export_rom for the file:line list).
%
% order 3 / 5 (ABI v3, default 5) adds e.poly: per function the Hermite cubic / quintic
% coefficients of every row, ntemp x (ntheta-1) x (order+1) (Uocp1: (ntheta-1) x
% (order+1)), in s = theta (ntheta-1) - i, from the handle's values and theta-derivatives
% (5-point finite differences of step 1e-4, one-sided at the ends so no call leaves
% [0, 1]); and e.Ea (1 x 5, J/mol, order Uocp dUocp k0 Rf Cdleff): a function found to be
% f(th,Tref) exp(Ea/R (1/Tref - 1/T)) gets its Ea and rows f(th, Tref), so the library
% evaluates it exactly at any T.  order 1: the v2 tables only.  The same steps as
% rom.py tabulate_handles (tested there against closed-form handles).
%
% nodes (ABI v4, default false; mpcekf_build_tables sets it): a function whose handle
% carries theta breakpoints (mpcekf_handle_nodes: interp1 / pchip / griddedInterpolant over
% measured data) also gets e.nodes.(name) = struct('x', 1 x m nodes, 'p', ntemp x (m-1) x
% (order+1)) (Uocp1: (m-1) x (order+1)): per segment the cubic through the handle at
% x_k + h (0, 1/3, 2/3, 1) in d = theta - x_k, zero-padded -- exact to rounding for any
% handle that is a cubic or less between its breakpoints (rom.py fit_segments).  The
% library then looks such a function up on its own nodes.
  if nargin < 4 || isempty(order), order = 5; end
  if nargin < 5 || isempty(Tref), Tref = 298.15; end
  if nargin < 6 || isempty(R), R = 8.3144621; end
  if nargin < 7 || isempty(nodes), nodes = false; end
  nt = numel(TK);  nth = numel(th);
  e = struct();
  e.theta0 = f.theta0();  e.theta100 = f.theta100();
  e.soc0 = arrayfun(@(T) f.soc(0, T), TK);
  e.soc100 = arrayfun(@(T) f.soc(1, T), TK);
  nDL = f.nDL();
  cdleff = @(t, T) f.Cdl(t, T)^(2 - nDL) * f.wDL(t, T)^(nDL - 1);   % OB_step.m:212-219
  fns = {@(t, T) f.Uocp(t, T), @(t, T) f.dUocp(t, T), @(t, T) f.k0(t, T), @(t, T) f.Rf(t, T), cdleff};
  names = {'Uocp', 'dUocp', 'k0', 'Rf', 'Cdleff'};
  for k = 1:5
    tab = zeros(nt, nth);
    for j = 1:nt
      tab(j, :) = arrayfun(@(t) fns{k}(t, TK(j)), th);
    end
    e.(names{k}) = tab;
  end
  try
    u1 = @(t) f.Uocp(t);                              % EKFmatsHandler.m:96, one argument
    u1(0.5);
  catch
    u1 = @(t) f.Uocp(t, Tref);                        % a handle that needs T: Tref
  end
  e.Uocp1 = arrayfun(u1, th);
  if order == 1, return; end
  assert(order == 3 || order == 5, 'mpcekf_tabulate_electrode: order 1, 3 or 5');
  h = 1 / (nth - 1);
  e.Ea = zeros(1, 5);
  e.poly = struct();
  for k = 1:5
    ea = detect_arrhenius(fns{k}, TK, Tref, R);
    e.Ea(k) = ea;
    P = zeros(nt, nth - 1, order + 1);
    for j = 1:nt
      Tr = TK(j);
      if ea ~= 0, Tr = Tref; end
      [y, d1, d2] = fd_derivs(@(t) fns{k}(t, Tr), th);
      P(j, :, :) = reshape(hermite(y, d1, d2, h, order), [1, nth - 1, order + 1]);
    end
    e.poly.(names{k}) = P;
  end
  [y, d1, d2] = fd_derivs(u1, th);
  e.poly.Uocp1 = hermite(y, d1, d2, h, order);
  if ~nodes, return; end
  % ABI v4 node tables; discovery on the cellData handles themselves (the wrappers above
  % capture the whole struct f)
  src = {{f.Uocp}, {f.dUocp}, {f.k0}, {f.Rf}, {f.Cdl, f.wDL}};
  e.nodes = struct();
  for k = 1:5
    xn = [];
    for q = 1:numel(src{k}), xn = union(xn, mpcekf_handle_nodes(src{k}{q})); end
    if numel(xn) < 2, continue; end
    P = zeros(nt, numel(xn) - 1, order + 1);
    for j = 1:nt
      Tr = TK(j);
      if e.Ea(k) ~= 0, Tr = Tref; end
      P(j, :, :) = reshape(fit_segments(@(t) fns{k}(t, Tr), xn, order + 1), [1, numel(xn) - 1, order + 1]);
    end
    e.nodes.(names{k}) = struct('x', xn, 'p', P);
  end
  xn = mpcekf_handle_nodes(f.Uocp);
  if numel(xn) >= 2
    e.nodes.Uocp1 = struct('x', xn, 'p', fit_segments(u1, xn, order + 1));
  end
end

function C = fit_segments(f, x, np)
  % rom.py fit_segments: the cubic through f at x_k + h (0, 1/3, 2/3, 1) per segment, in
  % d = theta - x_k; a segment whose quadratic and cubic terms are rounding noise is stored
  % as interp1's (y_k, (y_k+1 - y_k) / h); zero-padded to np coefficients
  V = inv(fliplr(vander([0, 1/3, 2/3, 1])));      % increasing powers of t = d / h
  m = numel(x);
  C = zeros(m - 1, np);
  for k = 1:m - 1
    a = x(k);  b = x(k + 1);  h = b - a;
    ys = [f(a); f(a + h / 3); f(a + 2 * h / 3); f(b)];
    q = V * ys;
    sc = max(max(abs(ys)), realmin);
    if abs(q(3)) <= 64 * eps * sc && abs(q(4)) <= 64 * eps * sc
      C(k, 1:2) = [ys(1), (ys(4) - ys(1)) / h];
    else
      C(k, 1:4) = [q(1), q(2) / h, q(3) / h^2, q(4) / h^3];
    end
  end
end

function [y, d1, d2] = fd_derivs(f, th)
  % rom.py fd_derivs: 5-point stencils, central inside [2e, 1 - 2e], one-sided at the ends
  e = 1e-4;
  y = arrayfun(f, th);  d1 = zeros(size(y));  d2 = zeros(size(y));
  for i = 1:numel(th)
    t = th(i);
    if t >= 2 * e && t <= 1 - 2 * e
      fm2 = f(t - 2 * e); fm1 = f(t - e); fp1 = f(t + e); fp2 = f(t + 2 * e);
      d1(i) = (-fp2 + 8 * fp1 - 8 * fm1 + fm2) / (12 * e);
      d2(i) = (-fp2 + 16 * fp1 - 30 * y(i) + 16 * fm1 - fm2) / (12 * e * e);
    else
      s = 1;  if t > 2 * e, s = -1; end
      g = arrayfun(@(k) f(t + s * k * e), 1:4);
      d1(i) = s * (-25 * y(i) + 48 * g(1) - 36 * g(2) + 16 * g(3) - 3 * g(4)) / (12 * e);
      d2(i) = (35 * y(i) - 104 * g(1) + 114 * g(2) - 56 * g(3) + 11 * g(4)) / (12 * e * e);
    end
  end
end

function C = hermite(y, m, k, h, order)
  % rom.py hermite_coefs: (ntheta-1) x (order+1) coefficients in s
  y = y(:);  a = h * m(:);  b = h * h * k(:);
  D = y(2:end) - y(1:end-1);  a0 = a(1:end-1);  a1 = a(2:end);  b0 = b(1:end-1);  b1 = b(2:end);
  if order == 3
    C = [y(1:end-1), a0, 3 * D - 2 * a0 - a1, a0 + a1 - 2 * D];
  else
    C = [y(1:end-1), a0, b0 / 2, 10 * D - 6 * a0 - 4 * a1 - (3 * b0 - b1) / 2, ...
         -15 * D + 8 * a0 + 7 * a1 + (3 * b0 - 2 * b1) / 2, 6 * D - 3 * (a0 + a1) - (b0 - b1) / 2];
  end
end

function ea = detect_arrhenius(f, TK, Tref, R)
  % rom.py detect_arrhenius: theta-independent ratio to Tref, log-linear in 1/T
  ea = 0;
  x = linspace(0.03, 0.97, 13);
  Ts = TK(abs(TK - Tref) > 1e-6);
  if isempty(Ts), return; end
  base = arrayfun(@(t) f(t, Tref), x);
  if any(~isfinite(base)) || any(base == 0), return; end
  eas = zeros(size(Ts));
  for j = 1:numel(Ts)
    r = arrayfun(@(t) f(t, Ts(j)), x) ./ base;
    if any(~isfinite(r)) || any(r <= 0) || (max(r) - min(r)) > 1e-10 * abs(r(1)), return; end
    eas(j) = R * log(mean(r)) / (1 / Tref - 1 / Ts(j));
  end
  if mean(eas) == 0 || max(abs(eas - mean(eas))) > 1e-8 * abs(mean(eas)), return; end
  ea = mean(eas);
end
