"""ctypes binding of the HIP engine library ``_tfg.so`` (C ABI: include/tfg.h).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc, gfx950).
There is no CPU fallback: when the library is missing, or no GPU is visible,
the engine raises instead of silently computing elsewhere.
"""

from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

__all__ = [
    "LIB_PATH", "NativeError", "TfgParams", "UNIFORM_DTYPE", "lib", "load", "check",
    "F32", "F64", "I32", "FIELD", "DIAG_NAMES",
]

LIB_PATH = Path(os.environ.get("TFG_LIB", Path(__file__).resolve().parent / "_tfg.so"))

ABI_VERSION = 8  # include/tfg.h TFG_ABI_VERSION
FLOW_ALL, FLOW_INTERIOR, FLOW_EDGES = 0, 1, 2  # tfg_ice_flow_step parts
PREV_DEPTH = -1  # tfg_get_field / tfg_set_field index: the fp64 previous-step depth (TFG_PREV_DEPTH)
F32, F64, I32 = 0, 1, 2
OK, ERR_ARG, ERR_HIP, ERR_STATE, ERR_DOMAIN = 0, 1, 2, 3, 4

# include/tfg.h field ids
FIELD = {
    "LW_in": 0, "P_air": 1, "Hum_sp": 2, "P": 3, "SW_in": 4, "T_air": 5, "uz": 6,
    "h_snow": 7, "h_swe": 8, "SM": 9, "h_ice": 10, "h_iwe": 11, "IM": 12, "M_total": 13, "RH": 14,
    "elev": 15, "slope": 16, "aspect": 17, "catch_id": 18,
    "Eccs": 19, "Ecci": 20, "albedo": 21, "n": 22, "window": 23, "Qc": 24,
}
DIAG_NAMES = ["vol_P", "vol_PR", "vol_PS", "vol_SM", "vol_IM", "P_max"]


class NativeError(RuntimeError):
    """A nonzero status from the C ABI; the message is tfg_last_error()."""

    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


class TfgParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in (
        "dt", "da_m2", "lat", "lon", "sin_lat", "cos_lat",
        "T_rain_snow", "dust_atten", "canopy_factor", "cloud_factor",
        "rho_air", "rho_snow", "rho_ice", "rho_H2O", "h_active_layer", "T0",
        "Cp_air", "Cp_ice", "Cp_snow", "g", "Lf", "eps", "kappa", "latent_heat_constant", "Lv",
        "sigma", "sea_level_p0", "uni_gas_const", "M_mass_air", "z0_air", "em_surf",
    )] + [("satterlund", ctypes.c_int32), ("ring_len", ctypes.c_int32), ("glens_A", ctypes.c_double)]


# tfg_uniforms, one record per time step (numpy structured dtype, C layout)
_U_D = ["th", "omega_th", "cos_wth", "sin_wth", "sin_d", "cos_d", "tan_d", "isc_e0", "m_opt",
        "k_et_flat", "flat_sr", "flat_ss"]
_U_F = ["cos_wth_f", "sin_wth_f", "omega_th_f", "tan_d_f", "kc_f", "ks_f", "k_et_flat_f",
        "tau_c0", "tau_c1", "gam_c0", "gam_c1", "pad_f"]
UNIFORM_DTYPE = np.dtype(
    [(n, "<f8") for n in _U_D] + [(n, "<f4") for n in _U_F]
    + [("frame", "<i4"), ("hist", "<i4"), ("slot", "<i4"), ("flat_dark", "<i4")]
)

_lib = None


def load() -> ctypes.CDLL:
    """Load and type the engine library (once).  Raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise ImportError(
            f"HIP engine library not found at {LIB_PATH}; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950). "
            "There is no CPU fallback."
        )
    # One HIP runtime per process.  The torch wheel bundles its own
    # libamdhip64 under the same soname as /opt/rocm's; if this library were
    # loaded first it would bind /opt/rocm's runtime, and a later
    # `import torch` would load a second runtime that then reports no GPU.
    # Importing torch first makes this library bind torch's runtime, which
    # every caller that also uses torch (bench, sharding, device-tensor I/O)
    # then shares.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(str(LIB_PATH))
    vp, i64, i32, dp = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.POINTER(ctypes.c_double)
    sigs = {
        "tfg_abi_version": ([], i32),
        "tfg_build_info": ([], ctypes.c_char_p),
        "tfg_device_count": ([ctypes.POINTER(ctypes.c_int)], i32),
        "tfg_create": ([ctypes.POINTER(TfgParams), i64, i64, i32, i32, i32, i32, i32, ctypes.POINTER(vp)], i32),
        "tfg_destroy": ([vp], i32),
        "tfg_set_stream": ([vp, vp], i32),
        "tfg_get_stream": ([vp, ctypes.POINTER(vp)], i32),
        "tfg_shared_stream": ([i32, ctypes.POINTER(vp)], i32),
        "tfg_set_field": ([vp, i32, i32, vp, i32, i64, i32], i32),
        "tfg_get_field": ([vp, i32, i32, vp, i32, i64, i32], i32),
        "tfg_init_state": ([vp], i32),
        "tfg_step": ([vp, vp, i64], i32),
        "tfg_set_fuse": ([vp, i32], i32),
        "tfg_get_diag": ([vp, dp, i32], i32),
        "tfg_reset_diag": ([vp], i32),
        "tfg_sync": ([vp], i32),
        "tfg_fill_synthetic": ([vp, ctypes.c_uint64, i64, i64, ctypes.POINTER(ctypes.c_float), i32], i32),
        "tfg_last_error": ([vp], ctypes.c_char_p),
        "tfg_terrain_from_dem": ([vp, ctypes.c_double, ctypes.c_double, vp, vp, i32, i32], i32),
        "tfg_ice_flow_edges": ([vp, dp, dp, i32], i32),
        "tfg_ice_flow_dmax": ([vp, ctypes.c_double, ctypes.c_double, dp, dp, i32, dp], i32),
        "tfg_ice_flow_step": ([vp, ctypes.c_double, ctypes.c_double, ctypes.c_double, dp, dp, i32, i32], i32),
        "tfg_ice_flow_run": ([vp, ctypes.c_double, ctypes.c_double, ctypes.c_double, i32], i32),
        "tfg_set_inputs": ([vp, i32, vp, i32, i64, i32], i32),
        "tfg_get_outputs": ([vp, i32, vp, i32, i64, i32], i32),
        "tfg_update": ([vp, i32, vp, i32, vp, vp, i32, i64], i32),
        "tfg_update_many": ([vp, i32, vp, vp, vp], i32),
        "tfg_conduction_edges": ([vp, dp, dp, i32], i32),
        "tfg_conduction_update": ([vp, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                   ctypes.c_double, dp, dp, i32], i32),
        "tfg_conduction_off": ([vp], i32),
        "tfg_nan_safe_launches": ([vp, ctypes.POINTER(i64)], i32),
        "tfg_set_step_form": ([vp, i32], i32),
        "tfg_set_flux": ([vp, i32], i32),
        "tfg_set_split": ([vp, i32], i32),
        "tfg_join": ([vp], i32),
        "tfg_get_split": ([vp, ctypes.POINTER(ctypes.c_int)], i32),
        "tfg_selftest_powers": ([i32, vp, i64, i32, vp], i32),
    }
    for name, (args, res) in sigs.items():
        if "TFG_LIB" in os.environ and not hasattr(L, name):
            continue  # an older library variant under same-box A/B (scripts/gpu_ab_same_box.sh)
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    # a same-box A/B may load an older library through TFG_LIB (one ABI back)
    older_ok = "TFG_LIB" in os.environ and L.tfg_abi_version() == ABI_VERSION - 1
    if L.tfg_abi_version() != ABI_VERSION and not older_ok:
        raise ImportError(f"{LIB_PATH}: ABI version {L.tfg_abi_version()} != {ABI_VERSION} (rebuild the library)")
    _lib = L
    return L


def elf_section(path: Path, name: str) -> bytes | None:
    """Bytes of one section of a 64-bit little-endian ELF file (None if absent)."""
    import struct

    data = Path(path).read_bytes()
    if data[:4] != b"\x7fELF" or data[4] != 2 or data[5] != 1:
        return None
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    sec = [struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize) for i in range(shnum)]
    stroff = sec[shstrndx][4]
    for sh_name, _typ, _flags, _addr, off, size, *_ in sec:
        end = data.index(b"\0", stroff + sh_name)
        if data[stroff + sh_name:end].decode() == name:
            return data[off:off + size]
    return None


def code_object_sha256(path: Path | None = None) -> str | None:
    """sha256 of the library's device code (its ``.hip_fatbin`` section: the
    gfx950 code objects of every kernel).  PMC traffic measured on one build is
    quoted for another only when these agree (bench.py roofline.traffic)."""
    import hashlib

    blob = elf_section(Path(path or LIB_PATH), ".hip_fatbin")
    return hashlib.sha256(blob).hexdigest() if blob else None


BENCH_KERNEL = "_ZN8tfg_kern7k_fusedIfLb0ELb0ELb0ELb0ELi1ELb0ELb0E"  # k_fused<float, false, false, false, false, 1, false, false>
BENCH_KERNEL_PREC = "_ZN8tfg_kern7k_fusedIfLb0ELb0ELb0ELb0ELi1ELb0ELb1E"  # ... the fp64-flux form (PREC = true)
BENCH_KERNEL_F64 = "_ZN8tfg_kern7k_fusedIdLb1ELb0ELb0ELb0ELi1ELb0ELb0E"  # k_fused<double, true, false, false, false, 1, false, false>


def gfx950_code_objects(path: Path | None = None) -> list[bytes]:
    """The gfx950 code objects (ELF) in the library's ``.hip_fatbin`` section:
    one clang offload bundle per translation unit, each holding a host entry
    and the device image (magic, entry count, then offset/size/triple per entry,
    offsets from the bundle's start)."""
    import struct

    blob = elf_section(Path(path or LIB_PATH), ".hip_fatbin") or b""
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    out, pos = [], blob.find(magic)
    while pos >= 0:
        n_entries, = struct.unpack_from("<Q", blob, pos + len(magic))
        o = pos + len(magic) + 8
        for _ in range(n_entries):
            off, size, tlen = struct.unpack_from("<QQQ", blob, o)
            triple = blob[o + 24:o + 24 + tlen].decode()
            o += 24 + tlen
            if triple.endswith("gfx950") and size:
                out.append(blob[pos + off:pos + off + size])
        pos = blob.find(magic, pos + 1)
    return out


def _elf_symbols(elf: bytes):
    """(name, value, size, type, section bytes, section address) of every sized
    symbol of a 64-bit ELF."""
    import struct

    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, _ = struct.unpack_from("<HHH", elf, 0x3A)
    sec = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + i * shentsize) for i in range(shnum)]
    syms = []
    for _name, typ, _fl, _addr, off, size, link, _info, _al, entsize in sec:
        if typ != 2:  # SHT_SYMTAB
            continue
        stroff = sec[link][4]
        for j in range(size // entsize):
            st_name, st_info, _other, st_shndx, st_value, st_size = struct.unpack_from("<IBBHQQ", elf, off + j * entsize)
            if st_size == 0 or st_shndx == 0 or st_shndx >= shnum:
                continue
            end = elf.index(b"\0", stroff + st_name)
            s = sec[st_shndx]
            syms.append((elf[stroff + st_name:end].decode(), st_value, st_size, st_info & 0xF, s[3], s[4]))
    return syms


def kernel_code_sha256(symbol_prefix: str = BENCH_KERNEL, path: Path | None = None) -> str | None:
    """sha256 of ONE kernel's gfx950 machine code: its instructions, its kernel
    descriptor (register counts, LDS, launch attributes) and, transitively, the
    code and data it reaches through PC-relative addressing (e.g. the
    __noinline__ dark_exact).  The PC-relative literals themselves are masked
    (s_getpc_b64 followed by s_add_u32 / s_addc_u32 with a literal) and so is
    the descriptor's entry offset: moving other kernels around in the code
    object, or changing them, leaves the hash alone, while any change to the
    instructions this kernel executes changes it.  bench.py quotes a PMC
    traffic profile only for the kernel code it was measured on."""
    import hashlib
    import struct

    for elf in gfx950_code_objects(path):
        syms = _elf_symbols(elf)
        entry = [s for s in syms if s[0].startswith(symbol_prefix) and s[3] == 2]  # STT_FUNC
        if not entry:
            continue
        by_addr = {s[1]: s for s in syms}
        h = hashlib.sha256()
        seen, todo = set(), [entry[0]]
        while todo:
            name, value, size, typ, sec_addr, sec_off = todo.pop(0)
            if value in seen:
                continue
            seen.add(value)
            code = bytearray(elf[sec_off + value - sec_addr:sec_off + value - sec_addr + size])
            if typ == 2:
                words = len(code) // 4
                for w in range(words - 4):
                    (ins,) = struct.unpack_from("<I", code, 4 * w)
                    if (ins & 0xFF80FF00) != 0xBE801C00:  # s_getpc_b64 sN (SOP1, opcode 28)
                        continue
                    pc = value + 4 * w + 4
                    (add,) = struct.unpack_from("<I", code, 4 * w + 4)
                    (addc,) = struct.unpack_from("<I", code, 4 * w + 12)
                    if (add >> 23) == 0x100 and (addc >> 23) == 0x104 and 0xFF in (add & 0xFF, (add >> 8) & 0xFF):
                        lo, = struct.unpack_from("<i", code, 4 * w + 8)
                        for t in (pc + lo, pc + lo - 4):  # @rel32@lo+4: the literal is target - pc + 4
                            if t in by_addr:
                                todo.append(by_addr[t])
                        struct.pack_into("<I", code, 4 * w + 8, 0)
                        struct.pack_into("<I", code, 4 * w + 16, 0)
            h.update(name.encode() + b"\0" + bytes(code))
        kd = [s for s in syms if s[0] == entry[0][0] + ".kd"]
        if kd:
            name, value, size, _t, sec_addr, sec_off = kd[0]
            d = bytearray(elf[sec_off + value - sec_addr:sec_off + value - sec_addr + size])
            d[16:24] = bytes(8)  # kernel_code_entry_byte_offset: where the code object put the kernel
            h.update(b"kd\0" + bytes(d))
        return h.hexdigest()
    return None


def lib() -> ctypes.CDLL:
    return load()


def check(rc: int, handle=None) -> None:
    if rc != OK:
        msg = lib().tfg_last_error(handle)
        raise NativeError(rc, (msg or b"").decode() or f"tfg error {rc}")


def exported_symbols() -> list[str]:
    """Names declared in include/tfg.h that the loaded library exports."""
    L = load()
    return [n for n in (
        "tfg_abi_version", "tfg_build_info", "tfg_device_count", "tfg_create", "tfg_destroy",
        "tfg_set_stream", "tfg_get_stream", "tfg_shared_stream", "tfg_set_field", "tfg_get_field", "tfg_init_state",
        "tfg_step", "tfg_set_fuse", "tfg_get_diag", "tfg_reset_diag", "tfg_sync",
        "tfg_fill_synthetic", "tfg_last_error", "tfg_terrain_from_dem", "tfg_ice_flow_edges", "tfg_ice_flow_dmax", "tfg_ice_flow_step", "tfg_ice_flow_run", "tfg_set_inputs", "tfg_get_outputs",
        "tfg_update", "tfg_update_many", "tfg_conduction_edges", "tfg_conduction_update", "tfg_conduction_off",
        "tfg_nan_safe_launches", "tfg_set_step_form", "tfg_set_flux", "tfg_set_split", "tfg_join", "tfg_get_split",
        "tfg_selftest_powers",
    ) if hasattr(L, n)]
