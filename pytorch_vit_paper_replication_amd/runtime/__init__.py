"""Runtime: flat parameter store (fp32 master / grad buffers + bf16 shadow) and hipGraph step capture."""
from .param_store import ParamStore, get_store, lookup_store

__all__ = ["ParamStore", "get_store", "lookup_store"]
