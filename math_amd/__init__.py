"""math_amd — MI355X-native reverse-mode autodiff hot path with Stan Math signatures.

The product is the header-only C++ layer (math_amd/include/stan/...) on top of
the device library libsmg_hip.so (C-ABI: include/smg_hip.h).  This Python
package only binds the C-ABI for tests and benchmarks (math_amd.hip).
"""
__all__ = ["hip"]
