"""cometbft_amd -- MI355X-native (gfx950) batch Ed25519 (and sr25519) verifier
for CometBFT's commit-verification hot path.

The product is libcmtverify.so (C ABI in include/cmtverify.h): HIP kernels that
verify one signature per lane, a host runtime (streams, pinned staging) and a
C++ replay of ValidatorSet.VerifyCommit* over device verdicts. This package is
the Python binding used by tests and bench.py; see DESIGN.md.
"""
from . import _native
from .crypto import (MODE_GO_STDLIB, MODE_ZIP215, BatchVerifier, Context, KeySet, PubKey, Sr25519BatchVerifier,
                     Sr25519PubKey, default_context, new_batch_verifier, pack_messages)

__all__ = ["MODE_GO_STDLIB", "MODE_ZIP215", "BatchVerifier", "Context", "KeySet", "PubKey", "Sr25519BatchVerifier",
           "Sr25519PubKey", "default_context", "new_batch_verifier", "pack_messages", "_native"]
