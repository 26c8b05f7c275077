/* Host stand-ins for the libbpf declarations mislo_probe.h uses: the map-definition macros
 * expand exactly as libbpf's do (so the map globals exist with their types), and the helpers
 * are implemented by probe_host.c over in-process hash maps and a record buffer. */
#ifndef MISLO_HOST_BPF_HELPERS_H
#define MISLO_HOST_BPF_HELPERS_H
#include <linux/types.h>

#define SEC(name) __attribute__((section(name), used))
#define __uint(name, val) int (*name)[val]
#define __type(name, val) __typeof__(val) *name
#ifndef __always_inline
#define __always_inline inline __attribute__((always_inline))
#endif

enum { BPF_ANY = 0, BPF_NOEXIST = 1, BPF_EXIST = 2 };
enum {
	BPF_MAP_TYPE_HASH = 1,
	BPF_MAP_TYPE_ARRAY = 2,
	BPF_MAP_TYPE_PERCPU_ARRAY = 6,
	BPF_MAP_TYPE_LRU_HASH = 9,
	BPF_MAP_TYPE_RINGBUF = 27,
};
#define LIBBPF_PIN_BY_NAME 1
#define BPF_RB_NO_WAKEUP 1

void *bpf_map_lookup_elem(void *map, const void *key);
long bpf_map_update_elem(void *map, const void *key, const void *value, __u64 flags);
long bpf_ringbuf_output(void *ringbuf, void *data, __u64 size, __u64 flags);
__u64 bpf_ktime_get_ns(void);
__u64 bpf_get_current_cgroup_id(void);
__u64 bpf_get_current_pid_tgid(void);
#endif
