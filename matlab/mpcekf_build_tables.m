function [R, err, ok, ntheta] = mpcekf_build_tables(ROM, TdegC, TC, opts)
% MPCEKF_BUILD_TABLES  The library's ROM struct (mpcekf_rom_struct) with electrode tables
% that meet the error budget -- the one table step mpcekf_export_rom and the OB_step
% drop-in share (rom.py export_electrodes is the same algorithm, tested on closed-form and
% lookup-table handles):
%
%  * every function whose handle carries theta breakpoints (mpcekf_handle_nodes) gets an
%    ABI v4 node table, kept when it meets its budget on its own (mpcekf_check_tables
%    'only'); the others use the uniform-grid Hermite quintics (ABI v3);
%  * without opts.ntheta, ntheta goes 257 -> 4097 (doubling) until every lookup meets the
%    budget over each electrode's operating theta range (0-100 % SOC widened by 0.04) at
%    opts.Teval;
%  * missing the budget at 4097: error 'mpcekf:budget' (opts.strict, the default), else
%    the last tables with ok = false.
%
% TdegC / TC as mpcekf_rom_struct (table temperatures, simulation temperatures).
% opts.Teval (K): where the budget is checked; default the table temperatures and their
% midpoints.  A function that is not Arrhenius-scaled in T (e.g. a two-term k0) is exact
% only at table temperatures, so a caller that knows its temperatures (the drop-in: the
% distinct Tc) passes them.  opts.order (5), opts.nodes (true), opts.ntheta ([]).
% err: mpcekf_check_tables' errors per electrode (err.neg, err.pos).
  if nargin < 2, TdegC = []; end
  if nargin < 3, TC = []; end
  if nargin < 4, opts = struct(); end
  order = getopt(opts, 'order', 5);
  nodes = getopt(opts, 'nodes', true);
  strict = getopt(opts, 'strict', true);
  Teval = getopt(opts, 'Teval', []);
  sizes = getopt(opts, 'ntheta', []);
  if isempty(sizes), sizes = [257, 513, 1025, 2049, 4097]; end
  fn = ROM.cellData.function;
  Tr = 298.15;
  if isfield(ROM.cellData.const, 'Tref'), Tr = ROM.cellData.const.Tref; end
  lim = @(g) [max(0, min(g.soc(0, Tr), g.soc(1, Tr)) - 0.04), min(1, max(g.soc(0, Tr), g.soc(1, Tr)) + 0.04)];
  sides = {'neg', 'pos'};
  for ntheta = sizes
    R = mpcekf_rom_struct(ROM, ntheta, TdegC, TC, order, nodes);
    th = linspace(0, 1, ntheta);
    ok = true;
    if isempty(Teval), Tev = []; else, Tev = Teval; end
    for s = 1:2
      f = fn.(sides{s});
      e = R.(sides{s});
      if isfield(e, 'nodes')   % a node table that misses its budget: the uniform grid instead
        for k = fieldnames(e.nodes)'
          [~, okk] = mpcekf_check_tables(f, e, th, R.tab_T_K, R.Tref, R.R, lim(f), Tev, k{1});
          if ~okk, e.nodes = rmfield(e.nodes, k{1}); end
        end
        if isempty(fieldnames(e.nodes)), e = rmfield(e, 'nodes'); end
        R.(sides{s}) = e;
      end
      [err.(sides{s}), oks] = mpcekf_check_tables(f, e, th, R.tab_T_K, R.Tref, R.R, lim(f), Tev);
      ok = ok && oks;
    end
    if ok, return; end
  end
  if strict
    error('mpcekf:budget', ['mpcekf_build_tables: the electrode tables miss the error budget at %d theta ' ...
          'points (neg Uocp %.3g V, k0 %.3g; pos Uocp %.3g V, k0 %.3g)'], ntheta, err.neg.Uocp, ...
          err.neg.k0_rel, err.pos.Uocp, err.pos.k0_rel);
  end
end

function v = getopt(s, name, def)
  if isfield(s, name) && ~isempty(s.(name)), v = s.(name); else, v = def; end
end
