function [A, C, D, names, xloc] = mpcekf_pack_models(ROM)
% MPCEKF_PACK_MODELS  ROM.ROMmdls(t,z).{A,C,D} -> dense arrays in the library's order.
%   A [nT, nZ, n+1]      diag(ROMmdls(t,z).A); the last (integrator) entry is 1
%                         (OB_step.m:165-186 setupBlend stacks exactly this diagonal)
%   C [nT, nZ, nz, n+1]  ROMmdls(t,z).C including its res0 column (initKF.m:91 drops it
%                         for the EKF; OB_step.m:88-163 keeps it for the plant)
%   D [nT, nZ, nz]       ROMmdls(t,z).D
%   names / xloc          ROM.tfData.names / ROM.tfData.xLoc (iterEKF.m:612-613)
% The per-model B is not exported: initKF.m:84-87 requires prod(B) == 1 and never
% stores it ("we know what it is"); the same three initKF.m checks (integrator,
% diagonal A, unit B; initKF.m:73-87) are applied here before anything is written.
  [nT, nZ] = size(ROM.ROMmdls);
  np1 = size(ROM.ROMmdls(1,1).A, 1);
  nz = size(ROM.ROMmdls(1,1).C, 1);
  A = zeros(nT, nZ, np1);  C = zeros(nT, nZ, nz, np1);  D = zeros(nT, nZ, nz);
  for t = 1:nT
    for z = 1:nZ
      M = ROM.ROMmdls(t, z);
      assert(isequal(size(M.A), [np1 np1]), 'mpcekf_pack_models: A(%d,%d) size', t, z);
      assert(M.A(end,end) == 1, 'mpcekf_pack_models: A(%d,%d) has no integrator state', t, z);
      assert(isequal(diag(diag(M.A)), M.A), 'mpcekf_pack_models: A(%d,%d) not diagonal', t, z);
      assert(prod(M.B) == 1, 'mpcekf_pack_models: B(%d,%d) not all unit values', t, z);
      A(t, z, :) = real(diag(M.A));                 % OB_step.m:176
      C(t, z, :, :) = M.C;
      D(t, z, :) = M.D(:);
    end
  end
  names = cellstr(ROM.tfData.names(:))';
  xloc = double(ROM.tfData.xLoc(:))';
end
