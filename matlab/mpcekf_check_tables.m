function [err, ok] = mpcekf_check_tables(f, e, th, TK, Tref, R, thlim, Teval, only)
% MPCEKF_CHECK_TABLES  Largest difference of the library's lookups (include/mpcekf.h: v2
% bilinear tables; the ABI v3 theta polynomials with the Arrhenius factor when e has a poly
% field; the ABI v4 node tables of the functions in e.nodes) from the original
% cellData.function handles, at 997 theta points in thlim (default [0.001, 0.999]) and at
% the temperatures Teval (K; default every table temperature and the midpoints between
% them -- a caller that knows the temperatures the simulation runs at, as the OB_step
% drop-in does, passes those), plus the deviation of soc(z,T) from the linear-in-z form the
% library assumes.  The library reproduces the lookups bit-for-bit, so this is the
% tabulation part of any real-MATLAB parity gap.  ok: every error within the budget
% (rom.py TABLE_BUDGET; a tenth of north_star's 1e-6 relative on phise ~ 0.08 V, into which
% Uocp_n enters directly, EKFmatsHandler.m:96).  only: one function name ('Uocp', 'dUocp',
% 'k0', 'Rf', 'Cdleff', or 'Uocp1' for the one-argument Uocp), as mpcekf_build_tables uses
% to test a node table on its own.  The same measure as rom.py table_errors.
  if nargin < 5 || isempty(Tref), Tref = 298.15; end
  if nargin < 6 || isempty(R), R = 8.3144621; end
  if nargin < 7 || isempty(thlim), thlim = [0.001, 0.999]; end
  if nargin < 8 || isempty(Teval), Teval = sort([TK, (TK(1:end-1) + TK(2:end)) / 2]); end
  if nargin < 9, only = ''; end
  x = linspace(thlim(1), thlim(2), 997);
  budget = struct('Uocp', 8e-9, 'dUocp_rel', 1e-7, 'k0_rel', 1e-9, 'Rf_rel', 1e-9, 'Cdleff_rel', 1e-3, 'soc_lin', 1e-12);
  err = struct('Uocp', 0, 'dUocp_rel', 0, 'k0_rel', 0, 'Rf_rel', 0, 'Cdleff_rel', 0, 'soc_lin', 0);
  nDL = f.nDL();
  want = @(nm) isempty(only) || strcmp(only, nm);
  for T = Teval(:)'
    if want('Uocp')
      err.Uocp = max(err.Uocp, max(abs(arrayfun(@(t) f.Uocp(t, T), x) - look(e, 'Uocp', 1, th, TK, x, T, Tref, R))));
    end
    if want('dUocp')
      d = arrayfun(@(t) f.dUocp(t, T), x);
      err.dUocp_rel = max(err.dUocp_rel, max(abs(d - look(e, 'dUocp', 2, th, TK, x, T, Tref, R)) ./ max(abs(d), eps)));
    end
    if want('k0')
      k = arrayfun(@(t) f.k0(t, T), x);
      err.k0_rel = max(err.k0_rel, max(abs(k - look(e, 'k0', 3, th, TK, x, T, Tref, R)) ./ abs(k)));
    end
    if want('Rf')
      r = arrayfun(@(t) f.Rf(t, T), x);
      err.Rf_rel = max(err.Rf_rel, max(abs(r - look(e, 'Rf', 4, th, TK, x, T, Tref, R)) ./ max(abs(r), eps)));
    end
    if want('Cdleff')
      c = arrayfun(@(t) f.Cdl(t, T)^(2 - nDL) * f.wDL(t, T)^(nDL - 1), x);
      err.Cdleff_rel = max(err.Cdleff_rel, max(abs(c - look(e, 'Cdleff', 5, th, TK, x, T, Tref, R)) ./ abs(c)));
    end
    if isempty(only)
      s0 = f.soc(0, T);  s1 = f.soc(1, T);
      err.soc_lin = max(err.soc_lin, max(abs(arrayfun(@(z) f.soc(z, T), x) - (s0 + x * (s1 - s0)))));
    end
  end
  if want('Uocp1')
    try
      u1 = arrayfun(@(t) f.Uocp(t), x);
    catch
      u1 = arrayfun(@(t) f.Uocp(t, Tref), x);
    end
    err.Uocp = max(err.Uocp, max(abs(u1 - look1(e, th, x))));
  end
  ok = true;
  for k = fieldnames(budget)'
    ok = ok && err.(k{1}) <= budget.(k{1});
  end
end

function v = horner(c, s)
  % c: numel(s) x ncoef, Horner c1 + s (c2 + s (...)) per column
  v = c(:, end).';
  for q = size(c, 2) - 1:-1:1, v = c(:, q).' + s .* v; end
end

function v = look1(e, th, x)
  % the one-argument Uocp: its node table, else the uniform polynomial, else the v2 table
  if isfield(e, 'nodes') && isfield(e.nodes, 'Uocp1')
    v = nodes_row(e.nodes.Uocp1.x, e.nodes.Uocp1.p, x);
  elseif isfield(e, 'poly') && ~isempty(e.poly)
    P = e.poly.Uocp1;
    nth = numel(th);
    xc = min(max(x, 0), 1);
    tt = xc * (nth - 1);
    i = min(floor(tt), nth - 2);
    v = horner(P(i + 1, :), tt - i);
  else
    v = interp1(th, e.Uocp1, min(max(x, 0), 1), 'linear');
  end
end

function v = nodes_row(xn, P, x)
  % ABI v4 row (include/mpcekf.h node / node_p): k = #{j in 2..m-1 : xn(j) <= theta}, d = theta - xn(k)
  xc = min(max(x, 0), 1);
  m = numel(xn);
  k = ones(size(xc));
  for j = 2:m - 1, k = k + (xn(j) <= xc); end
  v = horner(reshape(P(k, :), numel(xc), []), xc - xn(k));
end

function v = look(e, name, fk, th, TK, x, T, Tref, R)
  % the library's evaluation (include/mpcekf.h): theta rows, then T (clamped), then the
  % Arrhenius factor with the unclamped T
  t2 = e.(name);
  if isfield(t2, 'shape'), t2 = reshape(t2.data, t2.shape); end
  nth = numel(th);
  rows = zeros(numel(TK), numel(x));
  if isfield(e, 'nodes') && isfield(e.nodes, name)
    for j = 1:numel(TK)
      rows(j, :) = nodes_row(e.nodes.(name).x, reshape(e.nodes.(name).p(j, :, :), numel(e.nodes.(name).x) - 1, []), x);
    end
  elseif isfield(e, 'poly') && ~isempty(e.poly)
    P = e.poly.(name);
    if isfield(P, 'shape'), P = reshape(P.data, P.shape); end
    xc = min(max(x, 0), 1);
    tt = xc * (nth - 1);
    i = min(floor(tt), nth - 2);
    s = tt - i;
    for j = 1:numel(TK)
      c = reshape(P(j, i + 1, :), numel(x), []);   % numel(x) x (order+1)
      rows(j, :) = horner(c, s);
    end
  else
    rows = interp1(th, t2.', min(max(x, 0), 1), 'linear').';   % [ntemp, numel(x)]
  end
  if numel(TK) == 1
    v = rows;
  else
    Tc = min(max(T, TK(1)), TK(end));
    j = find(TK <= Tc, 1, 'last');  j = min(j, numel(TK) - 1);
    g = (Tc - TK(j)) / (TK(j + 1) - TK(j));
    v = rows(j, :) + g * (rows(j + 1, :) - rows(j, :));
  end
  if isfield(e, 'Ea') && ~isempty(e.Ea) && e.Ea(fk) ~= 0
    v = v * exp((e.Ea(fk) / R) * (1 / Tref - 1 / T));
  end
end
