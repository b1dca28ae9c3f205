"""Host-side physics support: the model clock (per-step uniform scalars) and
the named variable store.  Cell arithmetic lives in the HIP kernels."""
