"""Signal producers that feed the agent's rings.

* ``ebpf/`` -- CO-RE BPF programs for the 12 kernel signals (+ hello / minimal smoke and
  GPU-scheduler / RCCL-uprobe programs), all writing the 64-byte ``mislo_event`` record into
  one pinned BPF ring buffer, stamped with wall-clock ns in the kernel.
* ``rocprof/`` -- rocprofiler-sdk tool library (``libmislo_rocprof.so``) producing the four
  GPU signals from inside MI355X workloads without root.

``PROBES`` maps every catalogue signal to the object and programs that produce it (the
loader attaches per signal so the overhead guard can detach in shed order).
"""

import os

HERE = os.path.dirname(os.path.abspath(__file__))
EBPF_DIR = os.path.join(HERE, "ebpf")
ROCPROF_TOOL = os.path.join(HERE, "rocprof", "libmislo_rocprof.so")

# signal -> (producer, object, programs)
PROBES = {
    "dns_latency_ms": ("bpf", "dns_latency", ("dns_send", "dns_recv_ret")),
    "tcp_retransmits_total": ("bpf", "tcp_retransmit", ("retransmit",)),
    "runqueue_delay_ms": ("bpf", "runqueue_delay", ("rq_wakeup", "rq_wakeup_new", "rq_switch")),
    "connect_latency_ms": ("bpf", "connect_latency", ("connect4_enter", "connect4_exit", "connect6_enter",
                                                      "connect6_exit")),
    "connect_errors_total": ("bpf", "connect_latency", ("connect4_enter", "connect4_exit", "connect6_enter",
                                                        "connect6_exit")),
    "tls_handshake_ms": ("bpf", "tls_handshake", ("tls_enter", "tls_exit")),
    "tls_handshake_fail_total": ("bpf", "tls_handshake", ("tls_enter", "tls_exit")),
    "cpu_steal_pct": ("bpf", "cpu_steal", ("stat_wait",)),
    "cfs_throttled_ms": ("bpf", "cfs_throttle", ("cfs_throttle", "cfs_unthrottle")),
    "mem_reclaim_latency_ms": ("bpf", "mem_reclaim", ("reclaim_begin", "reclaim_end")),
    "disk_io_latency_ms": ("bpf", "disk_io_latency", ("rq_issue", "rq_complete")),
    "syscall_latency_ms": ("bpf", "syscall_latency", ("read_enter", "read_exit", "write_enter", "write_exit")),
    "gpu_queue_delay_ms": ("rocprof+bpf", "gpu_kfd", ("kfd_evict", "kfd_restore")),
    "hbm_pressure_pct": ("rocprof", "libmislo_rocprof", ()),
    "xgmi_link_latency_us": ("rocprof", "libmislo_rocprof", ()),
    "rccl_collective_ms": ("rocprof+bpf", "gpu_kfd", ("allreduce_enter", "allreduce_exit", "allgather_enter",
                                                      "allgather_exit", "reducescatter_enter",
                                                      "reducescatter_exit")),
    "hello_sys_enter_write_total": ("bpf", "hello_sys_enter_write", ("hello_write",)),
}
