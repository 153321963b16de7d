"""fabric_amd -- MI355X-native block-validation engine for Hyperledger Fabric's committer.

The engine itself is the C-ABI library fabric_amd/libfgv.so (include/fgv.h): HIP kernels for
gfx950 plus the C++ host side.  This Python package is a thin ctypes mirror of the
reference's interfaces (bccsp Hash/Verify, TxValidator.Validate, MVCC) for tests and bench.
"""
