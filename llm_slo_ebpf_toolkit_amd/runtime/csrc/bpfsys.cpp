#include "bpfsys.h"

#include <errno.h>
#include <linux/bpf.h>
#include <linux/perf_event.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cstring>

namespace mislo {

namespace {
inline int sys_bpf(int cmd, union bpf_attr* attr) {
  const long r = syscall(__NR_bpf, cmd, attr, sizeof(*attr));
  return r < 0 ? -errno : (int)r;
}
inline uint64_t ptr(const void* p) { return (uint64_t)(uintptr_t)p; }
}  // namespace

int bpf_obj_get(const std::string& path) {
  union bpf_attr a;
  std::memset(&a, 0, sizeof(a));
  a.pathname = ptr(path.c_str());
  return sys_bpf(BPF_OBJ_GET, &a);
}

int bpf_map_info(int fd, BpfMapInfo* out) {
  struct bpf_map_info info;
  std::memset(&info, 0, sizeof(info));
  union bpf_attr a;
  std::memset(&a, 0, sizeof(a));
  a.info.bpf_fd = (uint32_t)fd;
  a.info.info_len = sizeof(info);
  a.info.info = ptr(&info);
  const int r = sys_bpf(BPF_OBJ_GET_INFO_BY_FD, &a);
  if (r < 0) return r;
  out->type = info.type;
  out->id = info.id;
  out->key_size = info.key_size;
  out->value_size = info.value_size;
  out->max_entries = info.max_entries;
  out->map_flags = info.map_flags;
  out->name.assign(info.name, strnlen(info.name, sizeof(info.name)));
  return 0;
}

int bpf_map_find(const std::string& name, uint32_t value_size) {
  uint32_t id = 0;
  for (;;) {
    union bpf_attr a;
    std::memset(&a, 0, sizeof(a));
    a.start_id = id;
    if (sys_bpf(BPF_MAP_GET_NEXT_ID, &a) < 0) return -ENOENT;
    id = a.next_id;
    union bpf_attr b;
    std::memset(&b, 0, sizeof(b));
    b.map_id = id;
    const int fd = sys_bpf(BPF_MAP_GET_FD_BY_ID, &b);
    if (fd < 0) continue;  // gone meanwhile, or not permitted
    BpfMapInfo info;
    if (bpf_map_info(fd, &info) == 0 && info.name == name && (!value_size || info.value_size == value_size))
      return fd;
    close(fd);
  }
}

int bpf_map_lookup(int fd, const void* key, void* value) {
  union bpf_attr a;
  std::memset(&a, 0, sizeof(a));
  a.map_fd = (uint32_t)fd;
  a.key = ptr(key);
  a.value = ptr(value);
  return sys_bpf(BPF_MAP_LOOKUP_ELEM, &a);
}

int bpf_map_update(int fd, const void* key, const void* value, uint64_t flags) {
  union bpf_attr a;
  std::memset(&a, 0, sizeof(a));
  a.map_fd = (uint32_t)fd;
  a.key = ptr(key);
  a.value = ptr(value);
  a.flags = flags;
  return sys_bpf(BPF_MAP_UPDATE_ELEM, &a);
}

int bpf_map_delete(int fd, const void* key) {
  union bpf_attr a;
  std::memset(&a, 0, sizeof(a));
  a.map_fd = (uint32_t)fd;
  a.key = ptr(key);
  return sys_bpf(BPF_MAP_DELETE_ELEM, &a);
}

int bpf_map_next_key(int fd, const void* key, void* next) {
  union bpf_attr a;
  std::memset(&a, 0, sizeof(a));
  a.map_fd = (uint32_t)fd;
  a.key = ptr(key);
  a.next_key = ptr(next);
  return sys_bpf(BPF_MAP_GET_NEXT_KEY, &a);
}

int bpf_map_lookup_batch(int fd, void* in_batch, void* out_batch, void* keys, void* values, uint32_t* count) {
  union bpf_attr a;
  std::memset(&a, 0, sizeof(a));
  a.batch.in_batch = ptr(in_batch);
  a.batch.out_batch = ptr(out_batch);
  a.batch.keys = ptr(keys);
  a.batch.values = ptr(values);
  a.batch.count = *count;
  a.batch.map_fd = (uint32_t)fd;
  const int r = sys_bpf(BPF_MAP_LOOKUP_BATCH, &a);
  *count = a.batch.count;
  return r;
}

int perf_uprobe_open(const UprobeAttr& u) {
  struct perf_event_attr attr;
  std::memset(&attr, 0, sizeof(attr));
  attr.size = sizeof(attr);
  attr.type = u.pmu_type;
  attr.config = u.retprobe ? (1ull << u.retprobe_bit) : 0ull;
  attr.config1 = ptr(u.path.c_str());  // uprobe_path
  attr.config2 = u.offset;             // probe_offset
  // a system-wide uprobe is opened on one CPU: it fires for the binary on every CPU
  const long fd = syscall(__NR_perf_event_open, &attr, u.pid, u.pid == -1 ? 0 : -1, -1, PERF_FLAG_FD_CLOEXEC);
  return fd < 0 ? -errno : (int)fd;
}

int bpf_link_create_perf(int prog_fd, int perf_fd) {
  union bpf_attr a;
  std::memset(&a, 0, sizeof(a));
  a.link_create.prog_fd = (uint32_t)prog_fd;
  a.link_create.target_fd = (uint32_t)perf_fd;
  a.link_create.attach_type = BPF_PERF_EVENT;
  return sys_bpf(BPF_LINK_CREATE, &a);
}

int bpf_prog_run_on_cpu(int prog_fd, uint32_t cpu) {
  union bpf_attr a;
  std::memset(&a, 0, sizeof(a));
  a.test.prog_fd = (uint32_t)prog_fd;
  a.test.flags = BPF_F_TEST_RUN_ON_CPU;
  a.test.cpu = cpu;
  const int r = sys_bpf(BPF_PROG_TEST_RUN, &a);
  return r < 0 ? r : (int)a.test.retval;
}

int close_fd(int fd) { return close(fd) < 0 ? -errno : 0; }

bool bpf_syscall_available() {
  // BPF_PROG_LOAD-free probe: an invalid OBJ_GET answers -EPERM without privilege and
  // -ENOENT / -EINVAL with it
  union bpf_attr a;
  std::memset(&a, 0, sizeof(a));
  a.pathname = ptr("/sys/fs/bpf/.mislo-probe-nonexistent");
  const int r = sys_bpf(BPF_OBJ_GET, &a);
  return r != -EPERM && r != -ENOSYS;
}

}  // namespace mislo
