"""Mirror of the reference constants.py: LDPC(174,91) tables in the reference's 1-based layout.

Rebuilt from the generated CSR tables (_ldpc_tables.py, the same data the HIP kernels use).
"""
from . import _ldpc_tables as _T

FTX_LDPC_M = 83
FTX_LDPC_N = 174

kFTX_LDPC_Num_rows = [_T.CHK_START[m + 1] - _T.CHK_START[m] for m in range(FTX_LDPC_M)]
kFTX_LDPC_Nm = [[_T.EDGE_VAR[e] + 1 for e in range(_T.CHK_START[m], _T.CHK_START[m + 1])]
                + [0] * (7 - kFTX_LDPC_Num_rows[m]) for m in range(FTX_LDPC_M)]
_EDGE_CHK = {}
for _m in range(FTX_LDPC_M):
    for _e in range(_T.CHK_START[_m], _T.CHK_START[_m + 1]):
        _EDGE_CHK[_e] = _m
kFTX_LDPC_Mn = [[_EDGE_CHK[_T.VAR_EDGE[3 * n + j]] + 1 for j in range(3)] for n in range(FTX_LDPC_N)]
