"""tulips_amd — MI355X-native TULIPS Internet/TCP checksum path.

See DESIGN.md. The product is ``libtulips_csum.so`` (C ABI in
``include/tulips_csum.h``); ``tulips_amd.csum`` is its Python binding.
"""
from . import csum  # noqa: F401  (raises ImportError if the .so is missing)
from .csum import (COMPLEMENT, INET, RAW, TCP, CsumError, HostContext,  # noqa: F401
                   InvalidArgument, batch, batch_arena, batch_fixed, checksum,
                   icmpv4_checksum, ipv4_checksum, tcp_checksum, verify, verify_arena)

__all__ = ["csum", "RAW", "INET", "TCP", "COMPLEMENT", "CsumError",
           "InvalidArgument", "HostContext", "batch", "batch_arena", "batch_fixed",
           "verify", "verify_arena",
           "checksum", "ipv4_checksum", "icmpv4_checksum", "tcp_checksum"]
