function x = mpcekf_handle_nodes(h, depth)
% MPCEKF_HANDLE_NODES  The theta breakpoints a lookup-table handle carries: the union of
% every strictly ascending, finite, real numeric vector of >= 3 values inside [0, 1] that
% the handle captured -- functions(h).workspace{1}, recursing into captured handles,
% structs (e.g. a pchip pp's breaks), cells and griddedInterpolant grids.  [] for a
% closed-form handle.  A captured vector that is not a breakpoint set only refines the
% segments, which keeps a piecewise polynomial exact; mpcekf_build_tables checks the
% result against the handle anyway.  The same scan as rom.py discover_nodes.
%
% A ROM from the Plett-Trimboli toolchain typically defines, e.g.,
%   cellData.function.neg.Uocp = @(x,T) interp1(xU, U0, x) + (T - Tref) * interp1(xS, dS, x);
% whose workspace holds xU and xS (called at OB_step.m:313-314,337-340, iterEKF.m:362-363,
% 404-407 and EKFmatsHandler.m:84-85,96).
  if nargin < 2, depth = 0; end
  x = [];
  if depth > 8 || ~isa(h, 'function_handle'), return; end
  info = functions(h);
  if ~isfield(info, 'workspace') || isempty(info.workspace), return; end
  ws = info.workspace{1};
  x = scan(ws, depth + 1);
end

function x = scan(v, depth)
  x = [];
  if depth > 8, return; end
  if isa(v, 'function_handle')
    x = mpcekf_handle_nodes(v, depth);
  elseif isa(v, 'griddedInterpolant')
    g = v.GridVectors;
    x = scan(g{1}, depth + 1);
  elseif isstruct(v)
    for f = fieldnames(v)'
      for k = 1:numel(v)
        x = union(x, scan(v(k).(f{1}), depth + 1));
      end
    end
  elseif iscell(v)
    for k = 1:numel(v)
      x = union(x, scan(v{k}, depth + 1));
    end
  elseif isnumeric(v) && isreal(v) && isvector(v) && numel(v) >= 3
    v = double(v(:)');
    if all(isfinite(v)) && all(diff(v) > 0) && v(1) >= -1e-12 && v(end) <= 1 + 1e-12
      x = union(x, min(max(v, 0), 1));
    end
  end
  x = x(:)';
end
