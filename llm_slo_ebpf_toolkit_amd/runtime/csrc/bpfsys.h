// bpf(2) without libbpf: the handful of commands the agent needs to work with the maps the
// probes pinned under /sys/fs/bpf (REF pkg/collector/probe_manager.go:25-185 holds cilium/ebpf
// collections; NEW's loader pins, the agent only opens what is pinned):
//   BPF_OBJ_GET (open a pinned map), BPF_OBJ_GET_INFO_BY_FD (type / sizes / max_entries),
//   BPF_MAP_LOOKUP_ELEM / UPDATE_ELEM / DELETE_ELEM (mislo_cfg epochs and floors, mislo_pods),
//   BPF_MAP_LOOKUP_BATCH (bulk reads of the interning maps), BPF_MAP_GET_NEXT_KEY (fallback).
// Each call returns 0 / an fd, or -errno.
#pragma once

#include <cstdint>
#include <string>

namespace mislo {

struct BpfMapInfo {
  uint32_t type, id, key_size, value_size, max_entries, map_flags;
  std::string name;
};

int bpf_obj_get(const std::string& path);
int bpf_map_info(int fd, BpfMapInfo* out);
// The first loaded map named `name` (BPF object names: <= 15 chars) whose values are
// `value_size` bytes (0: any): an fd, or -ENOENT. Needs CAP_SYS_ADMIN (map ids). For maps
// a probe object keeps private (not pinned by the loader): gpu_kfd.bpf.c hip_activity.
int bpf_map_find(const std::string& name, uint32_t value_size);
int bpf_map_lookup(int fd, const void* key, void* value);
int bpf_map_update(int fd, const void* key, const void* value, uint64_t flags);
int bpf_map_delete(int fd, const void* key);
int bpf_map_next_key(int fd, const void* key, void* next);
// one batch step: *count in = capacity, out = entries read; in_batch null = from the start;
// returns 0, or -ENOENT at the end (entries of the last step are still valid)
int bpf_map_lookup_batch(int fd, void* in_batch, void* out_batch, void* keys, void* values, uint32_t* count);
bool bpf_syscall_available();  // probe: is bpf(2) permitted at all (root / CAP_BPF)

// Uprobe attachment without libbpf (the probes' uprobe programs are pinned by the loader; the
// agent attaches them to the binaries it resolves per process, collector/uprobes.py):
//   perf_event_open(PERF_TYPE = the uprobe PMU's dynamic type, config = retprobe bit,
//   config1 = binary path, config2 = file offset of the function, pid = -1, cpu = 0) -> fd,
//   then BPF_LINK_CREATE(prog fd, perf fd, BPF_PERF_EVENT) -> link fd (closing it detaches).
struct UprobeAttr {
  uint32_t pmu_type;      // /sys/bus/event_source/devices/uprobe/type
  uint32_t retprobe_bit;  // /sys/bus/event_source/devices/uprobe/format/retprobe ("config:N")
  bool retprobe;
  std::string path;       // the binary, as the agent sees it (/proc/<pid>/root/...)
  uint64_t offset;        // file offset of the probed instruction
  int pid;                // -1: every process mapping the binary
};
int perf_uprobe_open(const UprobeAttr& a);
int bpf_link_create_perf(int prog_fd, int perf_fd);
int close_fd(int fd);

// BPF_PROG_TEST_RUN of a raw_tp program on one CPU (BPF_F_TEST_RUN_ON_CPU: the kernel runs it
// there, in an IPI): the agent's window-cut flush of that CPU's staging batches
// (probes/ebpf/mislo_flush.bpf.c). The program's return value, or -errno.
int bpf_prog_run_on_cpu(int prog_fd, uint32_t cpu);

}  // namespace mislo
