"""The tie-resolved parity checker lives with the oracle (oracle/ties.py); re-exported for the tests."""
from oracle.ties import (TIE_TOL, TieResolvingHook, code_position, gpu_codes_by_prefix,  # noqa: F401
                         load_oracle_weight_codes, oracle_weight_codes, tie_check, tie_resolved_vit_check)
