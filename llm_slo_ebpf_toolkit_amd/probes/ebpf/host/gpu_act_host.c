/* Host build of gpu_kfd.bpf.c's HIP / ROCr call accounting (mislo_gpu_act.h, the code the
 * uprobes run) over in-process maps: replays a script of uprobe hits from stdin and prints every
 * process's mislo_hip_act, so tests/test_probes.py compares it with a model of the rules.
 *
 *   stdin:  SUBMIT <copy 0|1> <tgid> <tid> <now_ns>      hip_launch / hip_copy entry count
 *           ENTER  <kind> <tgid> <tid> <now_ns>          a timed call's entry (kind 0 sync, 1 copy, 2 wait)
 *           EXIT   <kind> <tgid> <tid> <now_ns>          its return
 *   stdout: <tgid> launches copies last_ns sync_ns syncs copy_ns wait_ns waits   (one line per process) */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <linux/types.h>

#ifndef __always_inline
#define __always_inline inline __attribute__((always_inline))
#endif
enum { BPF_ANY = 0, BPF_NOEXIST = 1, BPF_EXIST = 2 };

#include "mislo_record.h"

#define CAP 4096
struct slot {
	int used;
	__u64 key;
	unsigned char val[sizeof(struct mislo_hip_act)];
};
struct hmap {
	unsigned key_size, val_size;
	struct slot s[CAP];
};
static struct hmap act_t0 = {8, 8}, hip_activity = {4, sizeof(struct mislo_hip_act)};

static __u64 key_of(const struct hmap *m, const void *key)
{
	__u64 k = 0;
	memcpy(&k, key, m->key_size);
	return k;
}

static struct slot *find(struct hmap *m, __u64 k)
{
	for (int i = 0; i < CAP; ++i)
		if (m->s[i].used && m->s[i].key == k)
			return &m->s[i];
	return NULL;
}

void *bpf_map_lookup_elem(void *map, const void *key)
{
	struct hmap *m = map;
	struct slot *s = find(m, key_of(m, key));
	return s ? s->val : NULL;
}

long bpf_map_update_elem(void *map, const void *key, const void *value, __u64 flags)
{
	struct hmap *m = map;
	__u64 k = key_of(m, key);
	struct slot *s = find(m, k);
	if (s && flags == BPF_NOEXIST)
		return -17; /* -EEXIST */
	if (!s)
		for (int i = 0; i < CAP && !s; ++i)
			if (!m->s[i].used)
				s = &m->s[i];
	if (!s)
		return -7;
	s->used = 1;
	s->key = k;
	memcpy(s->val, value, m->val_size);
	return 0;
}

long bpf_map_delete_elem(void *map, const void *key)
{
	struct hmap *m = map;
	struct slot *s = find(m, key_of(m, key));
	if (!s)
		return -2;
	s->used = 0;
	return 0;
}

#include "mislo_gpu_act.h"

int main(void)
{
	char op[16];
	unsigned kind, tgid, tid;
	unsigned long long now;
	while (scanf("%15s %u %u %u %llu", op, &kind, &tgid, &tid, &now) == 5) {
		__u64 pt = ((__u64)tgid << 32) | tid;
		if (!strcmp(op, "SUBMIT"))
			mislo_act_submit(&hip_activity, pt, (int)kind, now);
		else if (!strcmp(op, "ENTER"))
			mislo_act_enter(&act_t0, pt, kind, now);
		else if (!strcmp(op, "EXIT"))
			mislo_act_exit(&act_t0, &hip_activity, pt, kind, now);
	}
	for (int i = 0; i < CAP; ++i) {
		if (!hip_activity.s[i].used)
			continue;
		const struct mislo_hip_act *a = (const void *)hip_activity.s[i].val;
		printf("%llu %llu %llu %llu %llu %llu %llu %llu %llu\n", (unsigned long long)hip_activity.s[i].key,
		       (unsigned long long)a->launches, (unsigned long long)a->copies, (unsigned long long)a->last_ns,
		       (unsigned long long)a->sync_ns, (unsigned long long)a->syncs, (unsigned long long)a->copy_ns,
		       (unsigned long long)a->wait_ns, (unsigned long long)a->waits);
	}
	return 0;
}
