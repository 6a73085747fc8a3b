"""mosrx — Python mirror of the MI355X rx classifier's C ABI (include/mosrx.h).

Thin ctypes binding over the in-tree ``libmosrx.so``; every call goes to the
HIP path.  There is no CPU fallback: when the library or a gfx950 GPU is
missing, ``Context()`` raises.

The names mirror mOS's receive path: ``classify`` is ProcessPacket
(core/src/eth_in.c:27) over a batch, records carry the verdict it returns plus
the raw ip_fast_csum / TCPCalcChecksum values and the GetRSSHash /
GetRSSCPUCore outputs (core/src/util.c:61-131).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG_DIR, "libmosrx.so")

RESULT_DTYPE = np.dtype([
    ("rss", "<u4"), ("ip_csum", "<u2"), ("tcp_csum", "<u2"), ("payloadlen", "<u2"),
    ("payload_off", "u1"), ("verdict", "i1"), ("reason", "u1"), ("queue", "u1"),
    ("tcp_flags", "u1"), ("ihl_doff", "u1"),
])
assert RESULT_DTYPE.itemsize == 16

REASONS = ["TCP_OK", "ARP", "NON_IPV4", "IP_SHORT", "IP_BADVER", "NOVERIFY_PASS", "IP_BADCSUM",
           "NOT_TCP", "TCP_SHORT", "TCP_BADCSUM", "TRUNCATED", "TCP_LEN_OK", "ICMP_LOCAL"]
R = {name: i for i, name in enumerate(REASONS)}
NREASON = len(REASONS)
MAX_LOCAL = 16

# mosrx_tcpinfo: pkt_info's TCP fields (FillPacketContextTCPInfo, tcp.c:258-270), host order
TCPINFO_DTYPE = np.dtype([("seq", "<u4"), ("ack_seq", "<u4"), ("window", "<u2"), ("ip_len", "<u2")])
assert TCPINFO_DTYPE.itemsize == 12
# mosrx_result8: the compact record (rss, reason, queue, verdict, tcp_flags)
RESULT8_DTYPE = np.dtype([("rss", "<u4"), ("reason", "u1"), ("queue", "u1"), ("verdict", "i1"),
                          ("tcp_flags", "u1")])
assert RESULT8_DTYPE.itemsize == 8
QUEUE_COMPACT = 1
HOST_PINNED = 1
KIND_SMALL, KIND_S13 = 0, 1


def shape_variant(kind: int, nt_tails: bool = True) -> int:
    """mosrx_set_variant value forcing a kernel shape (bits 2-6 = kind + 1; bit 1 = nt tails)."""
    return ((kind + 1) << 2) | (2 if nt_tails else 0)

QMAP_I40E, QMAP_IXGBE = 1, 0
TRACE_FW64, TRACE_S64, TRACE_M1500, TRACE_IMIX = 0, 1, 2, 3
TRACE_SEED_BASE = 0x6D4F5321   # MOSRX_TRACE_SEED: seed 0 selects TRACE_SEED_BASE + kind
WINDOW_END = 78       # MOSRX_WINDOW_END_SMALL: batches whose frames all fit take the SMALL tile

MS_KEY = bytes([0x6d, 0x5a, 0x56, 0xda, 0x25, 0x5b, 0x0e, 0xc2, 0x41, 0x67, 0x25, 0x3d, 0x43, 0xa3,
                0x8f, 0xb0, 0xd0, 0xca, 0x2b, 0xcb, 0xae, 0x7b, 0x30, 0xb4, 0x77, 0xcb, 0x2d, 0xa3,
                0x80, 0x30, 0xf2, 0x0c, 0x6a, 0x42, 0xb7, 0x3b, 0xbe, 0xac, 0x01, 0xfa])


class Params(C.Structure):
    """mosrx_params: the mOS stack state the verdict depends on."""
    _fields_ = [("num_msp", C.c_uint32), ("num_esp", C.c_uint32), ("forward", C.c_int32),
                ("num_queues", C.c_int32), ("queue_mode", C.c_int32), ("skip_tcp_csum", C.c_int32),
                ("rss_key_len", C.c_uint32), ("rss_key", C.c_uint8 * 52),
                ("num_local", C.c_uint32), ("local_ip", C.c_uint32 * MAX_LOCAL)]


def ip_raw(a: str) -> int:
    """Dotted quad -> the raw u32 mOS keeps in netdev ip_addr (network order, loaded little-endian)."""
    return int.from_bytes(bytes(int(x) for x in a.split(".")), "little")


class Batch(C.Structure):
    _fields_ = [("frames", C.c_void_p), ("frames_bytes", C.c_uint64), ("off", C.c_void_p),
                ("len", C.c_void_p), ("n", C.c_uint32), ("max_len", C.c_uint32),
                ("layout", C.c_uint32), ("off0", C.c_uint32), ("stride", C.c_uint32), ("reserved", C.c_uint32)]


BATCH_UNIFORM = 1   # mosrx_batch.layout: frame i expected at off0 + i * stride (a hint; off[] decides)


def uniform_layout(off: np.ndarray):
    """(off0, stride) when off[i] == off[0] + i * stride for every i (a fixed-stride
    packing, as a ring of equal-size frames has), else None."""
    off = np.asarray(off)
    if len(off) < 2:
        return None
    st = int(off[1]) - int(off[0])
    if st <= 0 or not (np.diff(off.astype(np.int64)) == st).all():
        return None
    return int(off[0]), st


def with_hint(b: Batch, hint) -> Batch:
    """b with the layout hint (off0, stride) set (None: no hint)."""
    if hint is not None:
        b.layout, b.off0, b.stride = BATCH_UNIFORM, int(hint[0]), int(hint[1])
    return b


BPF_INSN = np.dtype([("code", "<u2"), ("jt", "u1"), ("jf", "u1"), ("k", "<u4")])   # mosrx_bpf_insn
BPF_LEN_FRAME, BPF_LEN_IP = 0, 1
TX_IP_CSUM, TX_TCP_CSUM = 1 << 4, 1 << 5   # MOS_UPDATE_IP_CHKSUM / MOS_UPDATE_TCP_CHKSUM
OP_CLASSIFY, OP_CLASSIFY_FH, OP_BPF, OP_TX_CSUM, OP_CLASSIFY_BPF, OP_CLASSIFY_TI, OP_TX_CHECKS = 0, 1, 2, 3, 4, 5, 6
# include/mosrx.h mosrx_tx_check: the TX checks of a frame, the frame untouched
TX_CHECK_DTYPE = np.dtype([("ip_check", "<u2"), ("tcp_check", "<u2"), ("what", "u1"), ("ihl", "u1"),
                           ("pad", "<u2")])
BPF_MAX_PROGS = 32


class BpfProg(C.Structure):
    _fields_ = [("insns", C.c_void_p), ("len", C.c_uint32), ("len_mode", C.c_int32)]


class TraceC(C.Structure):
    _fields_ = [("frames", C.c_void_p), ("frames_bytes", C.c_uint64), ("off", C.c_void_p),
                ("len", C.c_void_p), ("n", C.c_uint32), ("max_len", C.c_uint32),
                ("caplen_sum", C.c_uint64)]


class RxStats(C.Structure):
    _fields_ = [("rx_packets", C.c_uint64), ("rx_bytes", C.c_uint64), ("rx_errors", C.c_uint64),
                ("rounds", C.c_uint64), ("batches", C.c_uint64), ("by_reason", C.c_uint64 * NREASON),
                ("recv_errors", C.c_uint64)]


class ModuleCfg(C.Structure):
    _fields_ = [("num_ifs", C.c_uint32), ("if_names", (C.c_char * 16) * 16),
                ("src", C.c_void_p * 16), ("batch", C.c_uint32), ("max_frame", C.c_uint32),
                ("gpu_base", C.c_int32), ("ngpu", C.c_int32), ("pipeline", C.c_int32),
                ("params", Params), ("bpf_progs", C.c_void_p), ("bpf_nprog", C.c_uint32),
                ("tx_batch", C.c_uint32), ("tcpinfo", C.c_int32), ("group", C.c_uint32),
                ("group_bytes", C.c_uint64), ("flowhash", C.c_int32), ("tx_csum", C.c_int32),
                ("numa", C.c_int32), ("compact", C.c_int32), ("group_max_us", C.c_uint32),
                ("direct_kb", C.c_uint32), ("direct_frames", C.c_uint32)]


class ModuleStats(C.Structure):
    _fields_ = [("rx_batches", C.c_uint64), ("rx_frames", C.c_uint64), ("tx_packets", C.c_uint64),
                ("tx_bytes", C.c_uint64), ("tx_errors", C.c_uint64), ("kernel_launches", C.c_uint64),
                ("kernel_ms", C.c_double), ("rx_drops", C.c_uint64),
                ("rx_reclassified", C.c_uint64), ("cpu", C.c_int32), ("device", C.c_int32),
                ("tx_csum_offloaded", C.c_uint64), ("cpu_node", C.c_int32), ("gpu_node", C.c_int32),
                ("rx_groups", C.c_uint64), ("max_group_frames", C.c_uint64), ("group_cap_frames", C.c_uint64),
                ("ns_per_frame_host", C.c_double), ("ns_per_byte_dev", C.c_double),
                ("rx_direct_groups", C.c_uint64)]


LAT_BINS = 1024


class LatencyProbe(C.Structure):
    """mosrx_latency_probe (include/mosrx_io_module.h): residency histograms of
    frames from a paced source, filled by the rx loop (RxLoopOpts.probe)."""
    _fields_ = [("src", C.c_void_p), ("t0_ns", C.c_uint64), ("ns_per_frame", C.c_double),
                ("skip", C.c_uint64), ("seen", C.c_uint64), ("recorded", C.c_uint64), ("batches", C.c_uint64),
                ("avail_max_ns", C.c_uint64), ("done_max_ns", C.c_uint64),
                ("avail_hist", C.c_uint64 * LAT_BINS), ("done_hist", C.c_uint64 * LAT_BINS)]

    @staticmethod
    def bin_ns(b: int) -> float:
        """The middle of histogram bin b, ns (16 bins per octave above 16 ns)."""
        if b < 16:
            return float(b)
        e, m = b // 16, b % 16
        return ((16 + m) + 0.5) * 2.0 ** (e - 4)

    def percentiles(self, which: str = "avail", ps=(50, 99, 99.9)) -> dict:
        h = np.array(getattr(self, which + "_hist")[:], dtype=np.float64)
        tot = h.sum()
        if tot == 0:
            return {}
        cum = np.cumsum(h) / tot
        return {f"p{p:g}_us": round(self.bin_ns(int(np.searchsorted(cum, p / 100.0))) / 1e3, 2) for p in ps}


class RxLoopOpts(C.Structure):
    _fields_ = [("max_pkts", C.c_uint64), ("idle_rounds", C.c_uint32), ("idle_us", C.c_uint32),
                ("max_us", C.c_uint64), ("probe", C.c_void_p)]


class AfpOpts(C.Structure):
    _fields_ = [("ring_blocks", C.c_uint32), ("retire_ms", C.c_uint32), ("fanout_group", C.c_uint32),
                ("copy", C.c_int32)]


class AfpInfo(C.Structure):
    _fields_ = [("zero_copy", C.c_int32), ("ring_bytes", C.c_uint64), ("dropped_outgoing", C.c_uint64),
                ("ring_packets", C.c_uint64), ("ring_drops", C.c_uint64)]


class Forwarder(C.Structure):
    _fields_ = [("iom", C.c_void_p), ("ctx", C.c_void_p), ("out_if", C.c_int32 * 16),
                ("forwarded", C.c_uint64), ("dropped", C.c_uint64),
                ("forward", C.c_int32), ("num_msp", C.c_uint32), ("listener", C.c_uint32)]


class MosrxError(OSError):
    pass


_lib = None


def build():
    """Compile libmosrx.so in-tree (hipcc --offload-arch=gfx950 + gcc)."""
    subprocess.check_call(["make", "-s", "-C", PKG_DIR])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MosrxError(2, f"{LIB_PATH} missing: run build() / `make -C {PKG_DIR}`")
        L = C.CDLL(LIB_PATH)
        P, U32, U64, I = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int
        sig = {
            "mosrx_abi_version": (I, []),
            "mosrx_strerror": (C.c_char_p, [I]),
            "mosrx_params_default": (None, [C.POINTER(Params)]),
            "mosrx_params_set_ms_key": (None, [C.POINTER(Params)]),
            "mosrx_open": (I, [I, C.POINTER(Params), C.POINTER(P)]),
            "mosrx_set_params": (I, [P, C.POINTER(Params)]),
            "mosrx_set_variant": (I, [P, I]),
            "mosrx_close": (None, [P]),
            "mosrx_classify_dev": (I, [P, C.POINTER(Batch), P, P]),
            "mosrx_classify_host": (I, [P, C.POINTER(Batch), P]),
            "mosrx_classify_dev_fh": (I, [P, C.POINTER(Batch), P, P, P]),
            "mosrx_classify_host_fh": (I, [P, C.POINTER(Batch), P, P]),
            "mosrx_classify_dev_ex": (I, [P, C.POINTER(Batch), P, P, P, P]),
            "mosrx_classify_host_ex": (I, [P, C.POINTER(Batch), P, P, P]),
            "mosrx_classify_host_submit": (I, [P, I, C.POINTER(Batch), P]),
            "mosrx_classify_host_wait": (I, [P, I]),
            "mosrx_last_counters": (I, [P, C.POINTER(U64)]),
            "mosrx_sync": (I, [P]),
            "mosrx_dev_alloc": (I, [P, C.c_size_t, C.POINTER(P)]),
            "mosrx_dev_free": (I, [P, P]),
            "mosrx_host_alloc": (I, [P, C.c_size_t, C.POINTER(P)]),
            "mosrx_host_free": (I, [P, P]),
            "mosrx_memcpy_h2d": (I, [P, P, P, C.c_size_t]),
            "mosrx_memcpy_d2h": (I, [P, P, P, C.c_size_t]),
            "mosrx_memcpy_h2d_pull": (I, [P, P, P, C.c_size_t]),
            "mosrx_stream": (P, [P]),
            "mosrx_time_dev": (I, [P, C.POINTER(Batch), U32, C.POINTER(P), U32, C.POINTER(C.c_float)]),
            "mosrx_time_dev_kernels": (I, [P, C.POINTER(Batch), U32, C.POINTER(P), U32, C.POINTER(C.c_float)]),
            "mosrx_device_sync": (I, [P]),
            "mosrx_time_op": (I, [P, I, I, C.POINTER(Batch), U32, C.POINTER(P), C.POINTER(P), U32, U32,
                                  C.POINTER(C.c_float), C.POINTER(C.c_float)]),
            "mosrx_time_dev_streams": (I, [P, C.POINTER(Batch), U32, C.POINTER(P), U32, U32, C.POINTER(C.c_float)]),
            "mosrx_time_op_dispatch": (I, [P, I, I, C.POINTER(Batch), U32, C.POINTER(P), C.POINTER(P), U32,
                                           C.POINTER(C.c_float)]),
            "mosrx_time_queue_dispatch": (I, [P, C.POINTER(P), U32, U32, C.POINTER(C.c_float)]),
            "mosrx_probe_read_bw": (I, [P, U64, U32, U32, C.POINTER(C.c_float)]),
            "mosrx_probe_stamp_floor": (I, [P, C.POINTER(Batch), U32, C.POINTER(C.c_float)]),
            "mosrx_queue_create": (I, [P, C.POINTER(Batch), U32, C.POINTER(P), C.POINTER(P)]),
            "mosrx_queue_run": (I, [P, P, P]),
            "mosrx_queue_destroy": (None, [P, P]),
            "mosrx_time_queue": (I, [P, C.POINTER(P), U32, U32, C.POINTER(C.c_float), C.POINTER(C.c_float)]),
            "mosrx_time_host": (I, [P, C.POINTER(Batch), U32, C.POINTER(P), U32, C.POINTER(C.c_float)]),
            "mosrx_rss_tables": (I, [C.c_char_p, U32, C.POINTER(U32)]),
            "mosrx_tx_csum_dev": (I, [P, C.POINTER(Batch), I, P]),
            "mosrx_tx_csum_host": (I, [P, C.POINTER(Batch), I]),
            "mosrx_tx_csum_dev_checks": (I, [P, C.POINTER(Batch), I, P, P]),
            "mosrx_bpf_check": (I, [P, U32]),
            "mosrx_bpf_set": (I, [P, C.POINTER(BpfProg), U32]),
            "mosrx_bpf_dev": (I, [P, C.POINTER(Batch), P, P]),
            "mosrx_bpf_host": (I, [P, C.POINTER(Batch), P]),
            "mosrx_bpf_set_engine": (I, [P, I]),
            "mosrx_bpf_engine": (I, [P]),
            "mosrx_bpf_jit_log": (C.c_char_p, [P]),
            "mosrx_bpf_jit_source": (I, [C.POINTER(BpfProg), U32, C.POINTER(P)]),
            "mosrx_bpf_jit_hook_source": (I, [C.POINTER(BpfProg), U32, C.POINTER(P)]),
            "mosrx_bpf_jit_compile": (I, [C.POINTER(BpfProg), U32, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
            "mosrx_bpf_jit_compile_fused": (I, [C.POINTER(BpfProg), U32, C.c_char_p, C.c_size_t,
                                                C.POINTER(C.c_size_t)]),
            "mosrx_classify_bpf_dev": (I, [P, C.POINTER(Batch), P, P, P]),
            "mosrx_bpf_fused": (I, [P]),
            "mosrx_classify_bpf_host": (I, [P, C.POINTER(Batch), P, P]),
            "mosrx_classify_bpf_host_submit": (I, [P, I, C.POINTER(Batch), P, P]),
            "mosrx_trace_gen": (I, [I, U32, U32, U64, C.POINTER(TraceC)]),
            "mosrx_trace_free": (None, [C.POINTER(TraceC)]),
            "mosrx_source_mem": (P, [P, P, P, U32, U32]),
            "mosrx_source_pcap": (P, [C.c_char_p, U32]),
            "mosrx_source_afpacket": (P, [C.c_char_p]),
            "mosrx_source_close": (None, [P]),
            "mosrx_source_next": (I, [P, P, U32]),
            "mosrx_source_fill": (I, [P, P, U64, P, P, U32, U32, C.POINTER(U64)]),
            "mosrx_source_borrow": (I, [P, U32, U32, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64), P, P]),
            "mosrx_source_give_back": (I, [P]),
            "mosrx_source_mem_set_mode": (I, [P, I]),
            "mosrx_gpu_module_cfg_default": (None, [C.POINTER(ModuleCfg)]),
            "mosrx_gpu_module_configure": (I, [C.POINTER(ModuleCfg)]),
            "mosrx_gpu_module_bind": (I, [P, I]),
            "mosrx_rx_loop": (I, [P, P, I, U64, P, P, C.POINTER(RxStats)]),
            "mosrx_rx_loop_ex": (I, [P, P, I, C.POINTER(RxLoopOpts), P, P, C.POINTER(RxStats)]),
            "mosrx_source_paced": (P, [P, C.c_double]),
            "mosrx_source_paced_info": (I, [P, C.POINTER(U64), C.POINTER(C.c_double), C.POINTER(U64)]),
            "mosrx_classify_host_ready": (I, [P, I]),
            "mosrx_classify_host_reserve": (I, [P, U64, U32]),
            "mosrx_set_counters": (I, [P, I]),
            "mosrx_set_direct": (I, [P, U64, U32]),
            "mosrx_slot_direct": (I, [P, I]),
            "mosrx_mos_forwards": (I, [P, I, U32, U32]),
            "mosrx_device_count": (I, []),
            "mosrx_classify_host_submit_ex": (I, [P, I, C.POINTER(Batch), P, P]),
            "mosrx_classify_host_group_submit": (I, [P, I, C.POINTER(Batch), U32, C.POINTER(P), C.POINTER(P)]),
            "mosrx_classify_host_group_submit_ex": (I, [P, I, C.POINTER(Batch), U32, C.POINTER(P), C.POINTER(P),
                                                        C.POINTER(P)]),
            "mosrx_set_timing": (I, [P, I]),
            "mosrx_last_kernel_ms": (I, [P, C.POINTER(C.c_float)]),
            "mosrx_source_afpacket_ex": (P, [C.c_char_p, C.POINTER(AfpOpts)]),
            "mosrx_source_afpacket_info": (I, [P, C.POINTER(AfpInfo)]),
            "mosrx_source_tpacket_v3": (P, [P, U32, U32]),
            "mosrx_source_send": (I, [P, P, U32]),
            "mosrx_source_tx_pcap": (I, [P, C.c_char_p]),
            "mosrx_source_tx_flush": (I, [P]),
            "mosrx_source_tx_stats": (I, [P, C.POINTER(U64), C.POINTER(U64), C.POINTER(U64)]),
            "mosrx_gpu_module_bind_source": (I, [I, I, P]),
            "mosrx_gpu_module_device_of": (I, [I, I]),
            "mosrx_gpu_module_stats_of": (I, [P, C.POINTER(ModuleStats)]),
            "mosrx_gpu_module_set_timing": (I, [P, I]),
            "mosrx_bpf_set_async": (I, [P, C.POINTER(BpfProg), U32]),
            "mosrx_bpf_wait": (I, [P]),
            "mosrx_bpf_pending": (I, [P]),
            "mosrx_classify_dev_compact": (I, [P, C.POINTER(Batch), P, P]),
            "mosrx_queue_create_ex": (I, [P, C.POINTER(Batch), U32, C.POINTER(P), C.POINTER(P), C.POINTER(P), I,
                                          C.POINTER(P)]),
            "mosrx_classify_host_group_submit_bpf": (I, [P, I, C.POINTER(Batch), U32, C.POINTER(P), C.POINTER(P),
                                                         C.POINTER(P)]),
            "mosrx_classify_host_group_submit_c8": (I, [P, I, C.POINTER(Batch), U32, C.POINTER(P), C.POINTER(P)]),
            "mosrx_classify_host_group_submit_bpf_c8": (I, [P, I, C.POINTER(Batch), U32, C.POINTER(P),
                                                            C.POINTER(P), C.POINTER(P)]),
            "mosrx_host_register": (I, [P, P, C.c_size_t, I]),
            "mosrx_host_unregister": (I, [P, P]),
            "mosrx_pci_numa_node": (I, [C.c_char_p]),
            "mosrx_cpu_numa_node": (I, [I]),
            "mosrx_gpu_numa_node": (I, [I]),
            "mosrx_numa_pick": (I, [I, C.POINTER(C.c_int), I]),
            "mosrx_topology_set_root": (I, [C.c_char_p]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
        _sigs.update(sig)
    return _lib


_sigs = {}


def module_lib(path: str):
    """Another build of gpu_module_func (e.g. the CPU test suite's build of the
    module over a stand-in for the GPU): a CDLL whose mosrx_gpu_module_*
    functions carry libmosrx's signatures, for GpuBackend(module_lib=...)."""
    lib()
    L = C.CDLL(path)
    for name, (res, args) in _sigs.items():
        if name.startswith("mosrx_gpu_module_"):
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
    return L


def _chk(rc: int, what: str):
    if rc:
        raise MosrxError(-rc, f"{what}: {lib().mosrx_strerror(rc).decode()}")


def default_params(**kw) -> Params:
    """simple_firewall's state (mosrx_params_default) with fields overridden; `key`
    = RSS key bytes, `local` = the netdevs' IPv4 addresses (dotted quads)."""
    p = Params()
    lib().mosrx_params_default(C.byref(p))
    key = kw.pop("key", None)
    local = kw.pop("local", None)
    if local is not None:
        if len(local) > MAX_LOCAL:
            raise ValueError("at most 16 local addresses")
        p.num_local = len(local)
        for i, a in enumerate(local):
            p.local_ip[i] = ip_raw(a) if isinstance(a, str) else int(a)
    for k, v in kw.items():
        setattr(p, k, v)
    if key is not None:
        if not 16 <= len(key) <= 52:
            raise ValueError("rss key must be 16..52 bytes")
        for i in range(52):
            p.rss_key[i] = key[i] if i < len(key) else 0
        p.rss_key_len = len(key)
    return p


BPF_ENGINE_INTERP, BPF_ENGINE_JIT = 0, 1


def _bpf_progs(progs):
    keep = [np.ascontiguousarray(i if i is not None else [], BPF_INSN) for i, _ in progs]
    arr = (BpfProg * max(1, len(progs)))()
    for j, ((_, mode), ins) in enumerate(zip(progs, keep)):
        arr[j].insns = ins.ctypes.data if len(ins) else None
        arr[j].len = len(ins)
        arr[j].len_mode = mode
    return arr, keep


def bpf_jit_source(progs) -> str:
    """mosrx_bpf_jit_source: the gfx950 kernel source generated for a program set."""
    arr, _keep = _bpf_progs(progs)
    out = C.c_void_p()
    _chk(lib().mosrx_bpf_jit_source(arr, len(progs), C.byref(out)), "mosrx_bpf_jit_source")
    try:
        return C.string_at(out.value).decode()
    finally:
        C.CDLL(None).free(out)


def bpf_jit_hook_source(progs) -> str:
    """mosrx_bpf_jit_hook_source: the fused kernel's generated hook for a program set."""
    arr, _keep = _bpf_progs(progs)
    out = C.c_void_p()
    _chk(lib().mosrx_bpf_jit_hook_source(arr, len(progs), C.byref(out)), "mosrx_bpf_jit_hook_source")
    try:
        return C.string_at(out.value).decode()
    finally:
        C.CDLL(None).free(out)


def bpf_jit_compile(progs):
    """mosrx_bpf_jit_compile: (rc, code-object bytes, hipRTC log); no GPU needed."""
    arr, _keep = _bpf_progs(progs)
    log = C.create_string_buffer(4096)
    sz = C.c_size_t(0)
    rc = lib().mosrx_bpf_jit_compile(arr, len(progs), log, len(log), C.byref(sz))
    return rc, int(sz.value), log.value.decode(errors="replace")


def bpf_jit_compile_fused(progs):
    """mosrx_bpf_jit_compile_fused: (rc, code-object bytes, hipRTC log) of the fused
    classify + BPF kernel; no GPU needed."""
    arr, _keep = _bpf_progs(progs)
    log = C.create_string_buffer(8192)
    sz = C.c_size_t(0)
    rc = lib().mosrx_bpf_jit_compile_fused(arr, len(progs), log, len(log), C.byref(sz))
    return rc, int(sz.value), log.value.decode(errors="replace")


def bpf_check(insns) -> int:
    """mosrx_bpf_check: 0 if mosrx_bpf_set would admit the program, else -errno."""
    ins = np.ascontiguousarray(insns, BPF_INSN)
    return lib().mosrx_bpf_check(ins.ctypes.data if len(ins) else None, len(ins))


class Trace:
    """A seeded synthetic batch (include/mosrx_trace.h) held as numpy arrays."""

    def __init__(self, kind: int, n: int, nflows: int = 1_000_000, seed: int = 0):
        t = TraceC()
        _chk(lib().mosrx_trace_gen(kind, n, nflows, seed, C.byref(t)), "mosrx_trace_gen")
        try:
            fb = int(t.frames_bytes)
            self.frames = np.ctypeslib.as_array(C.cast(t.frames, C.POINTER(C.c_uint8)), (fb + 64,)).copy()
            self.off = np.ctypeslib.as_array(C.cast(t.off, C.POINTER(C.c_uint32)), (t.n,)).copy() if t.n else np.zeros(0, np.uint32)
            self.len = np.ctypeslib.as_array(C.cast(t.len, C.POINTER(C.c_uint16)), (t.n,)).copy() if t.n else np.zeros(0, np.uint16)
            self.frames_bytes = fb
            self.n = int(t.n)
            self.max_len = int(t.max_len)
            self.caplen_sum = int(t.caplen_sum)
        finally:
            lib().mosrx_trace_free(C.byref(t))


class DevBuffer:
    """Device allocation owned by a Context (hipMalloc through the C ABI)."""

    def __init__(self, ctx: "Context", nbytes: int):
        self.ctx, self.nbytes = ctx, int(nbytes)
        p = C.c_void_p()
        _chk(lib().mosrx_dev_alloc(ctx.handle, max(self.nbytes, 1), C.byref(p)), "mosrx_dev_alloc")
        self.ptr = p.value

    def upload(self, arr: np.ndarray):
        a = np.ascontiguousarray(arr)
        assert a.nbytes <= self.nbytes
        _chk(lib().mosrx_memcpy_h2d(self.ctx.handle, self.ptr, a.ctypes.data, a.nbytes), "h2d")

    def download(self, arr: np.ndarray):
        assert arr.flags.c_contiguous and arr.nbytes <= self.nbytes
        _chk(lib().mosrx_memcpy_d2h(self.ctx.handle, arr.ctypes.data, self.ptr, arr.nbytes), "d2h")
        return arr

    def free(self):
        if self.ptr:
            lib().mosrx_dev_free(self.ctx.handle, self.ptr)
            self.ptr = None


class DevBatch:
    """A batch resident in HBM: frames + off + len, and its result buffer."""

    def __init__(self, ctx: "Context", frames: np.ndarray, off: np.ndarray, ln: np.ndarray,
                 frames_bytes: int | None = None, max_len: int | None = None, hint="auto"):
        frames = np.ascontiguousarray(frames, np.uint8)
        off = np.ascontiguousarray(off, np.uint32)
        ln = np.ascontiguousarray(ln, np.uint16)
        self.n = len(off)
        # the layout hint the batch is handed over with: "auto" = its own fixed
        # stride if it has one (the producer knows how it packed the frames),
        # None = none, or an explicit (off0, stride) -- tests give wrong ones
        self.hint = uniform_layout(off) if isinstance(hint, str) else hint
        self.frames_bytes = int(frames_bytes if frames_bytes is not None else len(frames))
        self.d_frames = DevBuffer(ctx, max(len(frames), 16))
        self.d_frames.upload(frames)
        self.d_off = DevBuffer(ctx, max(off.nbytes, 4))
        self.d_off.upload(off)
        self.d_len = DevBuffer(ctx, max(ln.nbytes, 2))
        self.d_len.upload(ln)
        self.d_out = DevBuffer(ctx, max(self.n * 16, 16))
        self.d_fhash = None   # allocated on the first classify_dev(..., flow_hash=True)
        self.d_tinfo = None   # allocated on the first classify_dev(..., tcpinfo=True)
        self.d_match = None   # allocated on the first bpf_dev
        self.d_out8 = None    # compact records, allocated on the first classify_dev_compact
        self.max_len = int(max_len if max_len is not None else (int(ln.max()) if self.n else 0))
        self.caplen_sum = int(ln.astype(np.uint64).sum())

    def batch(self) -> Batch:
        return with_hint(Batch(self.d_frames.ptr, self.frames_bytes, self.d_off.ptr, self.d_len.ptr, self.n,
                               self.max_len), self.hint)

    def results(self) -> np.ndarray:
        out = np.zeros(self.n, RESULT_DTYPE)
        if self.n:
            self.d_out.download(out)
        return out

    def frames(self, nbytes: int | None = None) -> np.ndarray:
        """The frame buffer as it is now in HBM (e.g. after tx_csum_dev)."""
        out = np.zeros(self.frames_bytes if nbytes is None else nbytes, np.uint8)
        return self.d_frames.download(out)

    def matches(self) -> np.ndarray:
        out = np.zeros(self.n, np.uint32)
        if self.n:
            self.d_match.download(out)
        return out

    def results8(self) -> np.ndarray:
        out = np.zeros(self.n, RESULT8_DTYPE)
        if self.n:
            self.d_out8.download(out)
        return out

    def flow_hashes(self) -> np.ndarray:
        out = np.zeros(self.n, np.uint32)
        if self.n:
            self.d_fhash.download(out)
        return out

    def tcpinfo(self) -> np.ndarray:
        out = np.zeros(self.n, TCPINFO_DTYPE)
        if self.n:
            self.d_tinfo.download(out)
        return out

    def free(self):
        for b in (self.d_frames, self.d_off, self.d_len, self.d_out, self.d_fhash, self.d_match, self.d_tinfo,
                  self.d_out8):
            if b is not None:
                b.free()


class Context:
    """mosrx_ctx: one per host thread, bound to one GPU."""

    def __init__(self, device: int = 0, params: Params | None = None):
        self.params = params or default_params()
        h = C.c_void_p()
        _chk(lib().mosrx_open(device, C.byref(self.params), C.byref(h)), "mosrx_open")
        self.handle = h.value
        self.device = device

    def close(self):
        if self.handle:
            lib().mosrx_close(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_variant(self, variant: int):
        _chk(lib().mosrx_set_variant(self.handle, variant), "mosrx_set_variant")

    def set_params(self, params: Params):
        _chk(lib().mosrx_set_params(self.handle, C.byref(params)), "mosrx_set_params")
        self.params = params

    # ---- end-to-end from host memory ----
    def classify_host(self, frames, off, ln, frames_bytes=None, max_len=0) -> np.ndarray:
        frames = np.ascontiguousarray(frames, np.uint8)
        off = np.ascontiguousarray(off, np.uint32)
        ln = np.ascontiguousarray(ln, np.uint16)
        out = np.zeros(len(off), RESULT_DTYPE)
        b = Batch(frames.ctypes.data, int(frames_bytes if frames_bytes is not None else len(frames)),
                  off.ctypes.data, ln.ctypes.data, len(off), max_len)
        _chk(lib().mosrx_classify_host(self.handle, C.byref(b), out.ctypes.data), "mosrx_classify_host")
        return out

    def classify_host_ex(self, frames, off, ln, frames_bytes=None, max_len=0):
        """(records, flow hashes, pkt_info TCP fields) of a host batch in one GPU pass."""
        frames = np.ascontiguousarray(frames, np.uint8)
        off = np.ascontiguousarray(off, np.uint32)
        ln = np.ascontiguousarray(ln, np.uint16)
        out = np.zeros(len(off), RESULT_DTYPE)
        fh = np.zeros(len(off), np.uint32)
        ti = np.zeros(len(off), TCPINFO_DTYPE)
        b = Batch(frames.ctypes.data, int(frames_bytes if frames_bytes is not None else len(frames)),
                  off.ctypes.data, ln.ctypes.data, len(off), max_len)
        _chk(lib().mosrx_classify_host_ex(self.handle, C.byref(b), out.ctypes.data, fh.ctypes.data,
                                          ti.ctypes.data), "mosrx_classify_host_ex")
        return out, fh, ti

    def classify_host_fh(self, frames, off, ln, frames_bytes=None, max_len=0):
        """Records plus the per-frame flow hash (HashFlow before the NUM_BINS mask)."""
        frames = np.ascontiguousarray(frames, np.uint8)
        off = np.ascontiguousarray(off, np.uint32)
        ln = np.ascontiguousarray(ln, np.uint16)
        out = np.zeros(len(off), RESULT_DTYPE)
        fh = np.zeros(len(off), np.uint32)
        b = Batch(frames.ctypes.data, int(frames_bytes if frames_bytes is not None else len(frames)),
                  off.ctypes.data, ln.ctypes.data, len(off), max_len)
        _chk(lib().mosrx_classify_host_fh(self.handle, C.byref(b), out.ctypes.data, fh.ctypes.data),
             "mosrx_classify_host_fh")
        return out, fh

    # ---- TX checksum rewrite (mosrx_tx_csum_*) ----
    def tx_csum_host(self, frames, off, ln, flags=TX_IP_CSUM | TX_TCP_CSUM, frames_bytes=None) -> np.ndarray:
        """A rewritten copy of `frames` (the input array is left as it is)."""
        out = np.array(frames, np.uint8, copy=True)
        off = np.ascontiguousarray(off, np.uint32)
        ln = np.ascontiguousarray(ln, np.uint16)
        b = Batch(out.ctypes.data, int(frames_bytes if frames_bytes is not None else len(out)),
                  off.ctypes.data, ln.ctypes.data, len(off), 0)
        _chk(lib().mosrx_tx_csum_host(self.handle, C.byref(b), flags), "mosrx_tx_csum_host")
        return out

    def tx_csum_dev_checks(self, db: "DevBatch", flags=TX_IP_CSUM | TX_TCP_CSUM) -> np.ndarray:
        """mosrx_tx_csum_dev_checks into the batch's record buffer: one
        TX_CHECK_DTYPE record per frame, the frames left as they are."""
        b = db.batch()
        _chk(lib().mosrx_tx_csum_dev_checks(self.handle, C.byref(b), flags, db.d_out.ptr, None),
             "mosrx_tx_csum_dev_checks")
        _chk(lib().mosrx_sync(self.handle), "mosrx_sync")
        raw = np.empty(max(db.n, 1) * 8, np.uint8)
        db.d_out.download(raw)
        return raw.view(TX_CHECK_DTYPE)[:db.n].copy()

    def tx_csum_dev(self, db: "DevBatch", flags=TX_IP_CSUM | TX_TCP_CSUM, sync: bool = True) -> None:
        b = db.batch()
        _chk(lib().mosrx_tx_csum_dev(self.handle, C.byref(b), flags, None), "mosrx_tx_csum_dev")
        if sync:
            _chk(lib().mosrx_sync(self.handle), "mosrx_sync")

    # ---- batched BPF (mosrx_bpf_*) ----
    def bpf_set(self, progs) -> None:
        """progs: list of (insns, len_mode); insns None/empty = no filter (matches)."""
        arr, _keep = _bpf_progs(progs)
        _chk(lib().mosrx_bpf_set(self.handle, arr, len(progs)), "mosrx_bpf_set")

    def bpf_set_async(self, progs) -> None:
        """mosrx_bpf_set_async: in effect at once (interpreter), compiled behind."""
        arr, _keep = _bpf_progs(progs)
        _chk(lib().mosrx_bpf_set_async(self.handle, arr, len(progs)), "mosrx_bpf_set_async")

    def bpf_wait(self) -> None:
        _chk(lib().mosrx_bpf_wait(self.handle), "mosrx_bpf_wait")

    def bpf_pending(self) -> bool:
        rc = lib().mosrx_bpf_pending(self.handle)
        if rc < 0:
            _chk(rc, "mosrx_bpf_pending")
        return rc == 1

    def bpf_set_engine(self, engine: int) -> None:
        """Engine of the next bpf_set: BPF_ENGINE_JIT (hipRTC-compiled set) or BPF_ENGINE_INTERP."""
        _chk(lib().mosrx_bpf_set_engine(self.handle, engine), "mosrx_bpf_set_engine")

    def bpf_engine(self) -> int:
        """Engine of the installed set."""
        return lib().mosrx_bpf_engine(self.handle)

    def bpf_fused(self) -> bool:
        """The installed set has a fused classify + BPF kernel."""
        return lib().mosrx_bpf_fused(self.handle) == 1

    def classify_bpf_dev(self, db: "DevBatch", sync: bool = True, stream: int | None = None) -> None:
        """Records into db.d_out and match masks into db.d_match in one pass."""
        if db.d_match is None:
            db.d_match = DevBuffer(self, max(db.n * 4, 4))
        b = db.batch()
        _chk(lib().mosrx_classify_bpf_dev(self.handle, C.byref(b), db.d_out.ptr, db.d_match.ptr, stream),
             "mosrx_classify_bpf_dev")
        if sync:
            _chk(lib().mosrx_sync(self.handle), "mosrx_sync")

    def classify_bpf_host(self, frames, off, ln, frames_bytes=None):
        """(records, match masks) of a host batch in one GPU pass."""
        frames = np.ascontiguousarray(frames, np.uint8)
        off = np.ascontiguousarray(off, np.uint32)
        ln = np.ascontiguousarray(ln, np.uint16)
        out = np.zeros(len(off), RESULT_DTYPE)
        match = np.zeros(len(off), np.uint32)
        b = Batch(frames.ctypes.data, int(frames_bytes if frames_bytes is not None else len(frames)),
                  off.ctypes.data, ln.ctypes.data, len(off), 0)
        _chk(lib().mosrx_classify_bpf_host(self.handle, C.byref(b), out.ctypes.data, match.ctypes.data),
             "mosrx_classify_bpf_host")
        return out, match

    def bpf_jit_log(self) -> str:
        return (lib().mosrx_bpf_jit_log(self.handle) or b"").decode(errors="replace")

    def bpf_host(self, frames, off, ln, frames_bytes=None) -> np.ndarray:
        frames = np.ascontiguousarray(frames, np.uint8)
        off = np.ascontiguousarray(off, np.uint32)
        ln = np.ascontiguousarray(ln, np.uint16)
        out = np.zeros(len(off), np.uint32)
        b = Batch(frames.ctypes.data, int(frames_bytes if frames_bytes is not None else len(frames)),
                  off.ctypes.data, ln.ctypes.data, len(off), 0)
        _chk(lib().mosrx_bpf_host(self.handle, C.byref(b), out.ctypes.data), "mosrx_bpf_host")
        return out

    def bpf_dev(self, db: "DevBatch", sync: bool = True, stream: int | None = None) -> None:
        """Match masks into db.d_match; `stream`: a caller's hipStream_t (None: the context's)."""
        if db.d_match is None:
            db.d_match = DevBuffer(self, max(db.n * 4, 4))
        b = db.batch()
        _chk(lib().mosrx_bpf_dev(self.handle, C.byref(b), db.d_match.ptr, stream), "mosrx_bpf_dev")
        if sync:
            _chk(lib().mosrx_sync(self.handle), "mosrx_sync")

    def last_counters(self) -> np.ndarray:
        c = (C.c_uint64 * NREASON)()
        _chk(lib().mosrx_last_counters(self.handle, c), "mosrx_last_counters")
        return np.array(c[:], np.uint64)

    # ---- device resident ----
    def upload(self, frames, off, ln, frames_bytes=None, max_len=None, hint="auto") -> DevBatch:
        return DevBatch(self, frames, off, ln, frames_bytes, max_len, hint)

    def classify_dev(self, db: DevBatch, sync: bool = True, flow_hash: bool = False, tcpinfo: bool = False) -> None:
        b = db.batch()
        if flow_hash and db.d_fhash is None:
            db.d_fhash = DevBuffer(self, max(db.n * 4, 4))
        if tcpinfo and db.d_tinfo is None:
            db.d_tinfo = DevBuffer(self, max(db.n * 12, 12))
        if tcpinfo:
            _chk(lib().mosrx_classify_dev_ex(self.handle, C.byref(b), db.d_out.ptr,
                                             db.d_fhash.ptr if flow_hash else None, db.d_tinfo.ptr, None),
                 "mosrx_classify_dev_ex")
        elif flow_hash:
            _chk(lib().mosrx_classify_dev_fh(self.handle, C.byref(b), db.d_out.ptr, db.d_fhash.ptr, None),
                 "mosrx_classify_dev_fh")
        else:
            _chk(lib().mosrx_classify_dev(self.handle, C.byref(b), db.d_out.ptr, None), "mosrx_classify_dev")
        if sync:
            _chk(lib().mosrx_sync(self.handle), "mosrx_sync")

    def classify_dev_compact(self, db: DevBatch, sync: bool = True) -> None:
        """8-byte records (mosrx_result8) into db.d_out8."""
        if db.d_out8 is None:
            db.d_out8 = DevBuffer(self, max(db.n * 8, 8))
        b = db.batch()
        _chk(lib().mosrx_classify_dev_compact(self.handle, C.byref(b), db.d_out8.ptr, None),
             "mosrx_classify_dev_compact")
        if sync:
            _chk(lib().mosrx_sync(self.handle), "mosrx_sync")

    def group_submit_bpf(self, slot: int, batches: list, outs: list, fhash: list | None, match: list) -> None:
        """mosrx_classify_host_group_submit_bpf over host batches (Batch structs);
        outs / fhash / match: lists of host pointers (wait with group_wait)."""
        n = len(batches)
        bs = (Batch * n)(*batches)
        o = (C.c_void_p * n)(*outs)
        f = (C.c_void_p * n)(*fhash) if fhash is not None else None
        m = (C.c_void_p * n)(*match)
        _chk(lib().mosrx_classify_host_group_submit_bpf(self.handle, slot, bs, n, o, f, m),
             "mosrx_classify_host_group_submit_bpf")

    def group_submit_c8(self, slot: int, batches: list, outs8: list, fhash: list | None = None,
                        match: list | None = None) -> None:
        """mosrx_classify_host_group_submit_c8 (match None) or _bpf_c8: 8-byte records
        into outs8 (host pointers), flow hashes and the installed set's masks."""
        n = len(batches)
        bs = (Batch * n)(*batches)
        o = (C.c_void_p * n)(*outs8)
        f = (C.c_void_p * n)(*fhash) if fhash is not None else None
        if match is None:
            _chk(lib().mosrx_classify_host_group_submit_c8(self.handle, slot, bs, n, o, f),
                 "mosrx_classify_host_group_submit_c8")
        else:
            m = (C.c_void_p * n)(*match)
            _chk(lib().mosrx_classify_host_group_submit_bpf_c8(self.handle, slot, bs, n, o, f, m),
                 "mosrx_classify_host_group_submit_bpf_c8")

    def group_submit_ex(self, slot: int, batches: list, outs: list, tinfo: list | None = None,
                        fhash: list | None = None) -> None:
        """mosrx_classify_host_group_submit_ex: 16-byte records into outs (host
        pointers), pkt_info TCP fields and flow hashes when given."""
        n = len(batches)
        bs = (Batch * n)(*batches)
        o = (C.c_void_p * n)(*outs)
        ti = (C.c_void_p * n)(*tinfo) if tinfo is not None else None
        f = (C.c_void_p * n)(*fhash) if fhash is not None else None
        _chk(lib().mosrx_classify_host_group_submit_ex(self.handle, slot, bs, n, o, ti, f),
             "mosrx_classify_host_group_submit_ex")

    def group_wait(self, slot: int) -> None:
        _chk(lib().mosrx_classify_host_wait(self.handle, slot), "mosrx_classify_host_wait")

    def set_direct(self, max_bytes: int, max_frames: int = 0xFFFFFFFF) -> None:
        """mosrx_set_direct: group submits of at most max_frames frames and max_bytes of
        pinned input run copy-free."""
        _chk(lib().mosrx_set_direct(self.handle, int(max_bytes), int(max_frames)), "mosrx_set_direct")

    def slot_direct(self, slot: int) -> bool:
        """mosrx_slot_direct: the slot's last group submit ran copy-free."""
        rc = lib().mosrx_slot_direct(self.handle, slot)
        if rc < 0:
            _chk(rc, "mosrx_slot_direct")
        return rc == 1

    def host_register(self, ptr: int, nbytes: int, flags: int = 0) -> None:
        _chk(lib().mosrx_host_register(self.handle, ptr, nbytes, flags), "mosrx_host_register")

    def host_unregister(self, ptr: int) -> None:
        _chk(lib().mosrx_host_unregister(self.handle, ptr), "mosrx_host_unregister")

    def queue_ex(self, dbs: list[DevBatch], flow_hash: bool = False, match: bool = False,
                 compact: bool = False) -> "Queue":
        return Queue(self, dbs, flow_hash=flow_hash, match=match, compact=compact)

    def time_dev(self, dbs: list[DevBatch], iters: int) -> float:
        bs = (Batch * len(dbs))(*[d.batch() for d in dbs])
        outs = (C.c_void_p * len(dbs))(*[d.d_out.ptr for d in dbs])
        ms = C.c_float()
        _chk(lib().mosrx_time_dev(self.handle, bs, len(dbs), outs, iters, C.byref(ms)), "mosrx_time_dev")
        return float(ms.value)

    def time_op(self, op: int, dbs: list[DevBatch], iters: int, nstreams: int = 1, arg: int = 0,
                total: bool = True, kernels: bool = True):
        """mosrx_time_op: (total ms over `iters` launches on `nstreams` streams,
        average single-launch ms); either is None when not requested."""
        for d in dbs:
            if op == OP_CLASSIFY_FH and d.d_fhash is None:
                d.d_fhash = DevBuffer(self, max(d.n * 4, 4))
            if op == OP_CLASSIFY_TI and d.d_tinfo is None:
                d.d_tinfo = DevBuffer(self, max(d.n * 12, 12))
            if op in (OP_BPF, OP_CLASSIFY_BPF) and d.d_match is None:
                d.d_match = DevBuffer(self, max(d.n * 4, 4))
        bs = (Batch * len(dbs))(*[d.batch() for d in dbs])
        outs = (C.c_void_p * len(dbs))(*[(d.d_match.ptr if op == OP_BPF else d.d_out.ptr) for d in dbs])
        aux = (C.c_void_p * len(dbs))(*[(d.d_match.ptr if op == OP_CLASSIFY_BPF else
                                         d.d_tinfo.ptr if op == OP_CLASSIFY_TI else
                                         (d.d_fhash.ptr if d.d_fhash else None)) for d in dbs])
        tot, avg = C.c_float(), C.c_float()
        _chk(lib().mosrx_time_op(self.handle, op, arg, bs, len(dbs), outs, aux, iters, nstreams,
                                 C.byref(tot) if total else None, C.byref(avg) if kernels else None),
             "mosrx_time_op")
        return (float(tot.value) if total else None), (float(avg.value) if kernels else None)

    def time_op_dispatch(self, op: int, dbs: list[DevBatch], iters: int, arg: int = 0):
        """mosrx_time_op_dispatch: the kernel's own average duration (ms), each
        launch stamped by its dispatch; None for an op that is not one kernel."""
        def ptr(buf):
            return buf.ptr if buf is not None else None
        bs = (Batch * len(dbs))(*[d.batch() for d in dbs])
        outs = (C.c_void_p * len(dbs))(*[(ptr(d.d_match) if op == OP_BPF else d.d_out.ptr) for d in dbs])
        aux = (C.c_void_p * len(dbs))(*[(ptr(d.d_match) if op == OP_CLASSIFY_BPF else
                                         ptr(d.d_tinfo) if op == OP_CLASSIFY_TI else
                                         ptr(d.d_fhash) if op == OP_CLASSIFY_FH else None) for d in dbs])
        ms = C.c_float()
        rc = lib().mosrx_time_op_dispatch(self.handle, op, arg, bs, len(dbs), outs, aux, iters, C.byref(ms))
        if rc == -95:   # -ENOTSUP: more than one launch per operation
            return None
        _chk(rc, "mosrx_time_op_dispatch")
        return float(ms.value)

    def time_dev_streams(self, dbs: list[DevBatch], iters: int, nstreams: int) -> float:
        """Total ms for `iters` launches spread round-robin over `nstreams` streams."""
        bs = (Batch * len(dbs))(*[d.batch() for d in dbs])
        outs = (C.c_void_p * len(dbs))(*[d.d_out.ptr for d in dbs])
        ms = C.c_float()
        _chk(lib().mosrx_time_dev_streams(self.handle, bs, len(dbs), outs, iters, nstreams, C.byref(ms)),
             "mosrx_time_dev_streams")
        return float(ms.value)

    def time_dev_kernels(self, dbs: list[DevBatch], iters: int) -> float:
        """Average kernel duration (ms), HIP events around every launch."""
        bs = (Batch * len(dbs))(*[d.batch() for d in dbs])
        outs = (C.c_void_p * len(dbs))(*[d.d_out.ptr for d in dbs])
        ms = C.c_float()
        _chk(lib().mosrx_time_dev_kernels(self.handle, bs, len(dbs), outs, iters, C.byref(ms)),
             "mosrx_time_dev_kernels")
        return float(ms.value)

    def queue(self, dbs: list[DevBatch]) -> "Queue":
        return Queue(self, dbs)

    def probe_read_bw(self, nbytes: int = 128 << 20, nbuf: int = 6, iters: int = 60) -> float:
        """Measured streaming-read ceiling (GB/s) of this device."""
        g = C.c_float()
        _chk(lib().mosrx_probe_read_bw(self.handle, nbytes, nbuf, iters, C.byref(g)), "mosrx_probe_read_bw")
        return float(g.value)

    def probe_stamp_floor(self, db: DevBatch, iters: int = 500) -> float:
        """mosrx_probe_stamp_floor: the dispatch-stamped duration (ms) of an empty
        kernel with the grid a classify launch of `db` has."""
        ms = C.c_float()
        b = db.batch()
        _chk(lib().mosrx_probe_stamp_floor(self.handle, C.byref(b), iters, C.byref(ms)), "mosrx_probe_stamp_floor")
        return float(ms.value)

    def device_sync(self):
        _chk(lib().mosrx_device_sync(self.handle), "mosrx_device_sync")

    def host_alloc(self, nbytes: int) -> tuple[int, np.ndarray]:
        p = C.c_void_p()
        _chk(lib().mosrx_host_alloc(self.handle, max(int(nbytes), 1), C.byref(p)), "mosrx_host_alloc")
        arr = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), (max(int(nbytes), 1),))
        return p.value, arr

    def host_free(self, ptr: int):
        lib().mosrx_host_free(self.handle, ptr)

    def time_host(self, batches: list[Batch], outs: list[int], iters: int) -> float:
        bs = (Batch * len(batches))(*batches)
        os_ = (C.c_void_p * len(outs))(*outs)
        ms = C.c_float()
        _chk(lib().mosrx_time_host(self.handle, bs, len(batches), os_, iters, C.byref(ms)), "mosrx_time_host")
        return float(ms.value)


class Queue:
    """mosrx_queue: one launch classifies every batch of the queue."""

    def __init__(self, ctx: Context, dbs: list[DevBatch], flow_hash: bool = False, match: bool = False,
                 compact: bool = False):
        self.ctx = ctx
        n = len(dbs)
        for d in dbs:
            if flow_hash and d.d_fhash is None:
                d.d_fhash = DevBuffer(ctx, max(d.n * 4, 4))
            if match and d.d_match is None:
                d.d_match = DevBuffer(ctx, max(d.n * 4, 4))
            if compact and d.d_out8 is None:
                d.d_out8 = DevBuffer(ctx, max(d.n * 8, 8))
        bs = (Batch * n)(*[d.batch() for d in dbs])
        outs = (C.c_void_p * n)(*[(d.d_out8.ptr if compact else d.d_out.ptr) for d in dbs])
        h = C.c_void_p()
        if not (flow_hash or match or compact):
            _chk(lib().mosrx_queue_create(ctx.handle, bs, n, outs, C.byref(h)), "mosrx_queue_create")
        else:
            fh = (C.c_void_p * n)(*[d.d_fhash.ptr for d in dbs]) if flow_hash else None
            mt = (C.c_void_p * n)(*[d.d_match.ptr for d in dbs]) if match else None
            _chk(lib().mosrx_queue_create_ex(ctx.handle, bs, n, outs, fh, mt, QUEUE_COMPACT if compact else 0,
                                             C.byref(h)), "mosrx_queue_create_ex")
        self.handle = h.value

    def run(self, sync: bool = True):
        _chk(lib().mosrx_queue_run(self.ctx.handle, self.handle, None), "mosrx_queue_run")
        if sync:
            _chk(lib().mosrx_sync(self.ctx.handle), "mosrx_sync")

    def time(self, iters: int, others: list["Queue"] = (), kernels: bool = True) -> tuple[float, float]:
        """(total ms of `iters` back-to-back launches cycling over self + others,
        average isolated-launch ms or None when `kernels` is False)."""
        qs = [self] + list(others)
        arr = (C.c_void_p * len(qs))(*[q.handle for q in qs])
        tot, kern = C.c_float(), C.c_float()
        _chk(lib().mosrx_time_queue(self.ctx.handle, arr, len(qs), iters, C.byref(tot),
                                    C.byref(kern) if kernels else None), "mosrx_time_queue")
        return float(tot.value), (float(kern.value) if kernels else None)

    def time_dispatch(self, iters: int, others: list["Queue"] = ()) -> float:
        """The queue kernel's own average duration (ms) over `iters` back-to-back
        launches cycling over self + others, each stamped by its dispatch."""
        qs = [self] + list(others)
        arr = (C.c_void_p * len(qs))(*[q.handle for q in qs])
        ms = C.c_float()
        _chk(lib().mosrx_time_queue_dispatch(self.ctx.handle, arr, len(qs), iters, C.byref(ms)),
             "mosrx_time_queue_dispatch")
        return float(ms.value)

    def destroy(self):
        if self.handle:
            lib().mosrx_queue_destroy(self.ctx.handle, self.handle)
            self.handle = None


def rss_tables(key: bytes) -> np.ndarray:
    out = (C.c_uint32 * 384)()
    _chk(lib().mosrx_rss_tables(key, len(key), out), "mosrx_rss_tables")
    return np.array(out[:], np.uint32)


# ---------------------------------------------------------------------------
# io_module_func backend (include/mosrx_io_module.h): gpu_module_func behind a
# raw-socket / loopback source, driven by the RunMainLoop-shaped rx loop.
# ---------------------------------------------------------------------------
_VOIDFN = C.CFUNCTYPE(None)
_CTXFN = C.CFUNCTYPE(None, C.c_void_p)
_IOCTLFN = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_int, C.c_int, C.c_void_p)
_RECVFN = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_int)
_RPTRFN = C.CFUNCTYPE(C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_uint16))
_WPTRFN = C.CFUNCTYPE(C.c_void_p, C.c_void_p, C.c_int, C.c_uint16)
_SENDFN = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_int)


class ResultC(C.Structure):
    """mosrx_result as a ctypes structure (RESULT_DTYPE's layout)."""
    _fields_ = [("rss", C.c_uint32), ("ip_csum", C.c_uint16), ("tcp_csum", C.c_uint16),
                ("payloadlen", C.c_uint16), ("payload_off", C.c_uint8), ("verdict", C.c_int8),
                ("reason", C.c_uint8), ("queue", C.c_uint8), ("tcp_flags", C.c_uint8), ("ihl_doff", C.c_uint8)]


# mosrx_pkt_fn: the rx loop's per-frame consumer (ProcessPacket's place)
_PKTFN = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_uint16, C.POINTER(ResultC))
PKT_TX_IP_CSUM, PKT_TX_TCP_CSUM = 0x01, 0x02
PKT_RX_RSS, DRV_NAME, PKT_RX_RESULTS, PKT_RX_MATCH = 0x03, 0x08, 0x10, 0x11
PKT_RX_TCPINFO, PKT_SET_PARAMS = 0x12, 0x13
PKT_RX_STATE, PKT_RX_RECLASSIFY, PKT_SET_BPF, PKT_RX_FHASH = 0x14, 0x15, 0x16, 0x17
PKT_RX_RESULTS8 = 0x18


class IoModuleFunc(C.Structure):
    """io_module_func (core/src/include/io_module.h:63-78): 14 function pointers."""
    _fields_ = [(n, C.c_void_p) for n in (
        "load_module_upper_half", "load_module_lower_half", "init_handle", "link_devices",
        "release_pkt", "get_wptr", "set_wptr", "send_pkts", "get_rptr", "get_nif", "recv_pkts",
        "select", "destroy_handle", "dev_ioctl")]


class RssInfo(C.Structure):
    _fields_ = [("pktidx", C.c_int8), ("hash_value", C.c_uint32)]


def gpu_module() -> IoModuleFunc:
    return IoModuleFunc.in_dll(lib(), "gpu_module_func")


class GpuBackend:
    """One mTCP-thread's view of gpu_module_func over in-memory / pcap sources."""

    def __init__(self, sources: list[int], params: Params | None = None, batch: int = 32768,
                 max_frame: int = 2048, pipeline: bool = True, cpu: int = 0, gpu_base: int = 0,
                 ngpu: int = 1, bpf=None, group: int = 1, tcpinfo: bool = False, tx_batch: int = 64,
                 timing: bool = False, flowhash: bool = False, tx_csum: bool = False, compact: bool = False,
                 group_bytes: int = 0, group_max_us: int = 0, direct_kb: int | None = None,
                 direct_frames: int | None = None, module_lib=None):
        self.L = L = module_lib or lib()
        cfg = ModuleCfg()
        L.mosrx_gpu_module_cfg_default(C.byref(cfg))
        cfg.num_ifs = len(sources)
        for i, s in enumerate(sources):
            cfg.src[i] = s
            cfg.if_names[i].value = f"gpu{i}".encode()
        cfg.batch, cfg.max_frame, cfg.pipeline = batch, max_frame, int(pipeline)
        cfg.gpu_base, cfg.ngpu = gpu_base, ngpu
        cfg.group, cfg.tcpinfo, cfg.tx_batch, cfg.flowhash = group, int(tcpinfo), tx_batch, int(flowhash)
        cfg.tx_csum = int(tx_csum)
        cfg.compact = int(compact)          # 8-byte records (results8), with or without filters
        cfg.group_bytes = group_bytes       # auto groups' frame bytes per launch (0: MOSRX_GROUP_AUTO_BYTES)
        cfg.group_max_us = group_max_us     # a group's latency budget (0: none)
        if direct_kb is not None:
            cfg.direct_kb = direct_kb       # copy-free groups up to this many KiB (0: none)
        if direct_frames is not None:
            cfg.direct_frames = direct_frames   # ... and up to this many frames
        if params is not None:
            cfg.params = params
        self.params = Params.from_buffer_copy(cfg.params)
        self._bpf = None
        if bpf:
            self._bpf = _bpf_progs(bpf)          # kept alive until init_handle has installed them
            cfg.bpf_progs = C.addressof(self._bpf[0])
            cfg.bpf_nprog = len(bpf)
        _chk(L.mosrx_gpu_module_configure(C.byref(cfg)), "mosrx_gpu_module_configure")
        self.nif = len(sources)
        self.sources = list(sources)
        self.m = IoModuleFunc.in_dll(L, "gpu_module_func")
        self._ctx_obj = C.c_uint64(0xC0DE0000 + cpu)      # stands in for struct mtcp_thread_context *
        self.ctx = C.addressof(self._ctx_obj)
        _chk(L.mosrx_gpu_module_bind(self.ctx, cpu), "mosrx_gpu_module_bind")
        _VOIDFN(self.m.load_module_upper_half)()
        _CTXFN(self.m.init_handle)(self.ctx)
        self._recv = _RECVFN(self.m.recv_pkts)
        self._rptr = _RPTRFN(self.m.get_rptr)
        self._ioctl = _IOCTLFN(self.m.dev_ioctl)
        self._wptr = _WPTRFN(self.m.get_wptr)
        self._send = _SENDFN(self.m.send_pkts)
        if timing:
            _chk(L.mosrx_gpu_module_set_timing(self.ctx, 1), "mosrx_gpu_module_set_timing")

    def recv_pkts(self, ifidx: int = 0) -> int:
        return self._recv(self.ctx, ifidx)

    def get_rptr(self, ifidx: int, index: int) -> bytes | None:
        ln = C.c_uint16()
        p = self._rptr(self.ctx, ifidx, index, C.byref(ln))
        return C.string_at(p, ln.value) if p else None

    def results(self, ifidx: int, n: int) -> np.ndarray:
        p = C.c_void_p()
        if self._ioctl(self.ctx, ifidx, PKT_RX_RESULTS, C.byref(p)):
            raise MosrxError(5, "dev_ioctl(MOSRX_PKT_RX_RESULTS)")
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), (n * 16,)).view(RESULT_DTYPE).copy()

    def results8(self, ifidx: int, n: int) -> np.ndarray:
        """The exposed batch's 8-byte records (a compact backend's batch without filters)."""
        p = C.c_void_p()
        if self._ioctl(self.ctx, ifidx, PKT_RX_RESULTS8, C.byref(p)):
            raise MosrxError(5, "dev_ioctl(MOSRX_PKT_RX_RESULTS8)")
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), (n * 8,)).view(RESULT8_DTYPE).copy()

    def matches(self, ifidx: int, n: int) -> np.ndarray:
        """dev_ioctl(MOSRX_PKT_RX_MATCH): the batch's BPF match masks."""
        p = C.c_void_p()
        if self._ioctl(self.ctx, ifidx, PKT_RX_MATCH, C.byref(p)):
            raise MosrxError(5, "dev_ioctl(MOSRX_PKT_RX_MATCH)")
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint32)), (n,)).copy()

    def fhashes(self, ifidx: int, n: int) -> np.ndarray:
        """dev_ioctl(MOSRX_PKT_RX_FHASH): the batch's flow-table hashes (cfg.flowhash)."""
        p = C.c_void_p()
        if self._ioctl(self.ctx, ifidx, PKT_RX_FHASH, C.byref(p)):
            raise MosrxError(5, "dev_ioctl(MOSRX_PKT_RX_FHASH)")
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint32)), (n,)).copy()

    def tcpinfo(self, ifidx: int, n: int) -> np.ndarray:
        """dev_ioctl(MOSRX_PKT_RX_TCPINFO): the batch's pkt_info TCP fields."""
        p = C.c_void_p()
        if self._ioctl(self.ctx, ifidx, PKT_RX_TCPINFO, C.byref(p)):
            raise MosrxError(5, "dev_ioctl(MOSRX_PKT_RX_TCPINFO)")
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), (n * 12,)).view(TCPINFO_DTYPE).copy()

    def set_params(self, ifidx: int, params: Params) -> int:
        """dev_ioctl(MOSRX_PKT_SET_PARAMS): the stack state changed (0 or -1)."""
        return self._ioctl(self.ctx, ifidx, PKT_SET_PARAMS, C.byref(params))

    def ioctl_raw(self, ifidx: int, cmd: int, argp) -> int:
        return self._ioctl(self.ctx, ifidx, cmd, argp)

    def send(self, ifidx: int, frame: bytes) -> None:
        """get_wptr + copy (EthernetOutput, eth_out.c:80-84): the frame waits for send_pkts."""
        p = self._wptr(self.ctx, ifidx, len(frame))
        if not p:
            raise MosrxError(5, "get_wptr")
        C.memmove(p, frame, len(frame))

    def send_offloaded(self, ifidx: int, frame: bytes, ip: bool, tcp: bool) -> tuple[int, int]:
        """get_wptr + copy, then mOS's TX checksum offload requests for the frame
        (ip_out.c:169-174, tcp_out.c:207-218: dev_ioctl with its IP header):
        the (PKT_TX_IP_CSUM, PKT_TX_TCP_CSUM) returns, None where not asked."""
        p = self._wptr(self.ctx, ifidx, len(frame))
        if not p:
            raise MosrxError(5, "get_wptr")
        C.memmove(p, frame, len(frame))
        iph = C.c_void_p(p + 14)
        ri = self._ioctl(self.ctx, ifidx, PKT_TX_IP_CSUM, iph) if ip else None
        rt = self._ioctl(self.ctx, ifidx, PKT_TX_TCP_CSUM, iph) if tcp else None
        return ri, rt

    def send_pkts(self, ifidx: int) -> int:
        return self._send(self.ctx, ifidx)

    def stats(self) -> ModuleStats:
        st = ModuleStats()
        _chk(self.L.mosrx_gpu_module_stats_of(self.ctx, C.byref(st)), "mosrx_gpu_module_stats_of")
        return st

    def forwarder(self, out_if: list[int], listener: bool = False) -> Forwarder:
        """A mosrx_forwarder for run_loop(forward=...): netdev i -> out_if[i], the
        frames mOS forwards under the backend's stack state (mosrx_mos_forwards);
        `listener`: an end-host socket listens (its orphans get a RST, not forwarded)."""
        f = Forwarder()
        f.iom = C.addressof(self.m)
        f.ctx = self.ctx
        for i in range(16):
            f.out_if[i] = out_if[i] if i < len(out_if) else -1
        f.forward, f.num_msp, f.listener = self.params.forward, self.params.num_msp, int(listener)
        return f

    def rss_of(self, ifidx: int, pktidx: int) -> int | None:
        ri = RssInfo(pktidx, 0)
        return None if self._ioctl(self.ctx, ifidx, PKT_RX_RSS, C.byref(ri)) else ri.hash_value

    def run_loop(self, max_pkts: int = 0, idle_rounds: int = 1, idle_us: int = 0, max_us: int = 0,
                 forward: Forwarder | None = None, probe: LatencyProbe | None = None) -> RxStats:
        """mosrx_rx_loop_ex over this backend; `forward`: the mosrx_forward_frame
        consumer; `probe`: the residency of a paced source's frames (RxLoopOpts.probe)."""
        st = RxStats()
        o = RxLoopOpts(max_pkts, idle_rounds, idle_us, max_us, C.addressof(probe) if probe is not None else None)
        fn, arg = None, None
        if forward is not None:
            fn, arg = C.cast(lib().mosrx_forward_frame, C.c_void_p), C.byref(forward)
        _chk(lib().mosrx_rx_loop_ex(C.addressof(self.m), self.ctx, self.nif, C.byref(o), fn, arg, C.byref(st)),
             "mosrx_rx_loop_ex")
        return st

    def close(self):
        if self.ctx:
            _CTXFN(self.m.destroy_handle)(self.ctx)
            self.ctx = None
            for s in self.sources:
                lib().mosrx_source_close(s)
            self.sources = []


SRC_BEST, SRC_FILL, SRC_PER_FRAME = 0, 1, 2


def paced_source(inner: int, rate_pps: float) -> int:
    """mosrx_source_paced: `inner`'s frames released at rate_pps (takes inner over)."""
    s = lib().mosrx_source_paced(inner, float(rate_pps))
    if not s:
        raise MosrxError(22, "mosrx_source_paced")
    return s


def mem_source(frames: np.ndarray, off: np.ndarray, ln: np.ndarray, loops: int = 1, mode: int = SRC_BEST) -> int:
    frames = np.ascontiguousarray(frames, np.uint8)
    off = np.ascontiguousarray(off, np.uint32)
    ln = np.ascontiguousarray(ln, np.uint16)
    s = lib().mosrx_source_mem(frames.ctypes.data, off.ctypes.data, ln.ctypes.data, len(off), loops)
    if not s:
        raise MosrxError(12, "mosrx_source_mem")
    if mode != SRC_BEST:
        _chk(lib().mosrx_source_mem_set_mode(s, mode), "mosrx_source_mem_set_mode")
    return s


def afpacket_source(ifname: str, ring_blocks: int = 8, retire_ms: int = 1, fanout_group: int = 0,
                    copy: bool = False) -> int:
    """mosrx_source_afpacket_ex (TPACKET_V3 ring; needs CAP_NET_RAW)."""
    o = AfpOpts(ring_blocks, retire_ms, fanout_group, int(copy))
    s = lib().mosrx_source_afpacket_ex(ifname.encode(), C.byref(o))
    if not s:
        raise MosrxError(1, f"mosrx_source_afpacket_ex({ifname})")
    return s


def afpacket_info(src: int) -> AfpInfo:
    i = AfpInfo()
    _chk(lib().mosrx_source_afpacket_info(src, C.byref(i)), "mosrx_source_afpacket_info")
    return i


def source_tx_pcap(src: int, path: str | None) -> None:
    _chk(lib().mosrx_source_tx_pcap(src, path.encode() if path else None), "mosrx_source_tx_pcap")


def source_send(src: int, frame: bytes) -> int:
    return lib().mosrx_source_send(src, frame, len(frame))


def source_tx_stats(src: int) -> tuple[int, int, int]:
    a, b, c = C.c_uint64(), C.c_uint64(), C.c_uint64()
    _chk(lib().mosrx_source_tx_stats(src, C.byref(a), C.byref(b), C.byref(c)), "mosrx_source_tx_stats")
    return a.value, b.value, c.value


def source_borrow(src, max_n: int, max_frame: int = 65535):
    """One zero-copy run of the source (mosrx_source_borrow): (frames as bytes
    objects, the run's base address, off, len), or None when nothing is ready.
    The run stays valid until source_give_back."""
    off = np.zeros(max(1, max_n), np.uint32)
    ln = np.zeros(max(1, max_n), np.uint16)
    base, nbytes = C.c_void_p(), C.c_uint64()
    n = lib().mosrx_source_borrow(src, max_n, max_frame, C.byref(base), C.byref(nbytes),
                                  off.ctypes.data, ln.ctypes.data)
    _chk(min(n, 0), "mosrx_source_borrow")
    if n == 0:
        return None
    frames = [C.string_at(base.value + int(o), int(l)) for o, l in zip(off[:n], ln[:n])]
    return frames, base.value, off[:n].copy(), ln[:n].copy()


def source_give_back(src) -> None:
    _chk(lib().mosrx_source_give_back(src), "mosrx_source_give_back")


def read_pcap(path: str) -> list[bytes]:
    """Frames of a classic pcap file through the library's own reader (mosrx_source_pcap)."""
    s = lib().mosrx_source_pcap(path.encode(), 1)
    if not s:
        raise MosrxError(2, f"mosrx_source_pcap({path})")
    buf = np.zeros(65536, np.uint8)
    out = []
    try:
        while True:
            n = lib().mosrx_source_next(s, buf.ctypes.data, len(buf))
            if n <= 0:
                return out
            out.append(bytes(buf[:n]))
    finally:
        lib().mosrx_source_close(s)


def _sysfs_props(path: str) -> dict:
    out = {}
    try:
        with open(path) as fh:
            for line in fh:
                k, _, v = line.strip().partition(" ")
                if v.strip().lstrip("-").isdigit():
                    out[k] = int(v)
    except OSError:
        pass
    return out


def _parse_cpulist(text: str) -> list[int]:
    cpus = []
    for part in text.strip().split(","):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        cpus += list(range(int(lo), int(hi or lo) + 1))
    return cpus


def gpu_numa_cpus(device: int, root: str = "/"):
    """(PCI address, NUMA node, that node's cores) of HIP device `device`, read from
    sysfs without touching the GPU (so a rank can bind itself before its first HIP
    call): the KFD topology's GPU nodes in order -- HIP's device order -- less those
    ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES hide, the GPU's PCI numa_node, the
    node's cpulist.  None when any of it is unknown."""
    base = os.path.join(root, "sys", "class", "kfd", "kfd", "topology", "nodes")
    try:
        ids = sorted(int(d) for d in os.listdir(base) if d.isdigit())
    except OSError:
        return None
    gpus = []
    for k in ids:
        pr = _sysfs_props(os.path.join(base, str(k), "properties"))
        if pr.get("simd_count", 0) > 0 and "location_id" in pr:
            loc = pr["location_id"]
            gpus.append(f"{pr.get('domain', 0):04x}:{(loc >> 8) & 0xFF:02x}:{(loc >> 3) & 0x1F:02x}.{loc & 7:x}")
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v:
            try:
                gpus = [gpus[int(x)] for x in v.split(",") if x.strip()]
            except (ValueError, IndexError):
                return None
    if not 0 <= device < len(gpus):
        return None
    bdf = gpus[device]
    try:
        with open(os.path.join(root, "sys", "bus", "pci", "devices", bdf, "numa_node")) as fh:
            node = int(fh.read().strip())
        with open(os.path.join(root, "sys", "devices", "system", "node", f"node{node}", "cpulist")) as fh:
            cpus = _parse_cpulist(fh.read())
    except (OSError, ValueError):
        return None
    return (bdf, node, cpus) if node >= 0 and cpus else None


def bind_to_gpu_node(device: int, root: str = "/") -> dict:
    """Bind the calling process to the cores of device's NUMA node (those it may
    run on), as mOS binds each mTCP thread to its core's node (cpu.c:56-87).
    Call before the first GPU call; never re-execs.  Returns what was done."""
    info = gpu_numa_cpus(device, root)
    if not info:
        return {"device": device, "bound": False, "why": "topology unknown"}
    bdf, node, cpus = info
    allowed = os.sched_getaffinity(0)
    mine = sorted(set(cpus) & allowed)
    if not mine:
        return {"device": device, "pci": bdf, "node": node, "bound": False,
                "why": f"none of node {node}'s cores in this process's affinity"}
    if set(mine) != allowed:
        os.sched_setaffinity(0, mine)
    return {"device": device, "pci": bdf, "node": node, "bound": True, "cpus": len(mine)}


def shard_plan(nbatches: int, world: int, rank: int) -> list[int]:
    """Round-robin split of a job's batches over GPUs: batch b -> GPU b % world.

    No exchange step exists between GPUs, so the plan is the whole multi-GPU protocol:
    each rank classifies its own batches; results land in disjoint slices."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    return list(range(rank, nbatches, world))


def split_batches(frames: np.ndarray, off: np.ndarray, ln: np.ndarray, batch: int):
    """Cut a packed trace into consecutive batches of `batch` frames (views re-based
    so every batch is self-contained: its own frames buffer and offsets)."""
    out = []
    for s in range(0, len(off), batch):
        o, l = off[s:s + batch], ln[s:s + batch]
        lo = int(o.min()) & ~15 if len(o) else 0
        hi = int((o.astype(np.uint64) + l).max()) if len(o) else 0
        out.append((frames[lo:hi + 64], (o - lo).astype(np.uint32), l.copy(), hi - lo))
    return out
