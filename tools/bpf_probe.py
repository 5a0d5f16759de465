"""Can this host run the eBPF restatement (BPF_PROG_TEST_RUN) as the current user?
Usage: python tools/bpf_probe.py"""
import os

try:
    print("unprivileged_bpf_disabled =", open("/proc/sys/kernel/unprivileged_bpf_disabled").read().strip())
except OSError as e:
    print("sysctl unreadable:", e)
try:
    print("bpf_jit_enable =", open("/proc/sys/net/core/bpf_jit_enable").read().strip())
except OSError as e:
    print("jit sysctl unreadable:", e)
print("uid", os.getuid(), "cpu_count", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))
