/* Host build of the probe plumbing (probe_host.c): the few kernel typedefs mislo_probe.h
 * needs. The BPF build uses the real vmlinux.h (bpftool btf dump, probes/ebpf/Makefile). */
#ifndef MISLO_HOST_VMLINUX_H
#define MISLO_HOST_VMLINUX_H
#include <linux/types.h>
#endif
