"""Drop-in `bls.FastAggregateVerify` (reference call site sync-protocol.md:464).

Semantics of upstream `eth2spec.utils.bls.FastAggregateVerify` with the py_ecc backend (the IETF
BLS draft's POP ciphersuite, `BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_`): every pubkey is
KeyValidated (decodes, is not the identity, lies in G1), the aggregate must not be the identity,
the signature must decode and lie in G2, then e(PK_agg, H(m)) == e(G1, sig); any malformed input
gives False (the eth2spec wrapper turns exceptions into False); an empty pubkey list gives False.
All arithmetic runs in the HIP kernels of liblcv.so.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np

from . import runtime
from .device import Verifier

bls_active = True


def FastAggregateVerify(pubkeys: Sequence[bytes], message: bytes, signature: bytes,
                        verifier: Optional[Verifier] = None) -> bool:
    if not bls_active:
        return True
    try:
        pks = [bytes(p) for p in pubkeys]
        msg, sig = bytes(message), bytes(signature)
    except Exception:
        return False
    if len(pks) == 0 or len(sig) != 96 or any(len(p) != 48 for p in pks):
        return False
    v = verifier if verifier is not None else runtime.default_verifier()
    # any key count (tables of 512 keys, slice aggregates summed on device) and any message length
    return v.fast_aggregate_verify(pks, msg, sig)


def FastAggregateVerifyBatch(committees: np.ndarray, committee_id: np.ndarray, bits: np.ndarray, messages: np.ndarray,
                             signatures: np.ndarray, verifier: Optional[Verifier] = None) -> np.ndarray:
    """Batched form: item i verifies the participants (bits[i]) of committees[committee_id[i]]."""
    v = verifier if verifier is not None else runtime.default_verifier()
    return v.fast_aggregate_verify_batch(committees, committee_id, bits, messages, signatures)
