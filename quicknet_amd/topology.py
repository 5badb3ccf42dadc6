"""Host topology for bench.py's rank launcher, read from sysfs with no HIP call.

The launching parent of `bench.py --gpus N` must not touch the GPU before it starts its rank
processes (a process that has initialised HIP must not be the parent of GPU work here), and
`torch.cuda.device_count()` can fall back to hipGetDeviceCount when amdsmi is unavailable.
So the parent counts devices from the KFD topology instead:

  /sys/class/kfd/kfd/topology/nodes/<id>/properties   one node per CPU socket and per GPU;
      GPU nodes have a non-zero gfx_target_version, plus location_id (PCI bus<<8|dev<<3|fn)
      and domain, which name the device's PCI function.

ROCr enumerates its GPU agents in KFD node order; ROCR_VISIBLE_DEVICES filters that list (by
index or by `GPU-<unique_id hex>`), and HIP_VISIBLE_DEVICES (or CUDA_VISIBLE_DEVICES) then
filters what ROCr left, so HIP device i is the i-th entry after both filters.

Each rank binds itself (before importing torch, so every thread it starts inherits the mask)
to the CPUs of its GPU's NUMA node -- /sys/bus/pci/devices/<bdf>/numa_node and local_cpulist
-- intersected with the CPUs it may run on, so the pinned host batches of the host-to-host
legs are first touched on the node the GPU's PCIe link hangs off.

Nothing here is on the codec path; SURVEY.md 8(e): groups partition across GPUs with no
collective (module/rs.c:582-586).
"""
import os

KFD_NODES = "sys/class/kfd/kfd/topology/nodes"
# the sysfs root the functions read by default; tests point it at a fake tree
SYSFS = os.environ.get("QFEC_SYSFS_ROOT", "/")
PCI_DEVICES = "sys/bus/pci/devices"
_UNREADABLE = 0  # KFD nodes the last kfd_gpus() call could not read


def _read(path):
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return None


def _props(path):
    txt = _read(path)
    if txt is None:
        return None
    out = {}
    for line in txt.splitlines():
        parts = line.split()
        if len(parts) == 2:
            try:
                out[parts[0]] = int(parts[1])
            except ValueError:
                pass
    return out


def parse_cpulist(s):
    """'0-3,8,10-11' -> {0,1,2,3,8,10,11}."""
    cpus = set()
    for part in (s or "").strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            cpus.update(range(int(a), int(b) + 1))
        else:
            cpus.add(int(part))
    return cpus


def kfd_gpus(sysfs=None):
    """GPU nodes of the KFD topology in node order, or None when the topology is unreadable."""
    sysfs = SYSFS if sysfs is None else sysfs
    root = os.path.join(sysfs, KFD_NODES)
    try:
        ids = sorted(int(x) for x in os.listdir(root) if x.isdigit())
    except OSError:
        return None
    gpus = []
    global _UNREADABLE
    _UNREADABLE = 0
    for i in ids:
        p = _props(os.path.join(root, str(i), "properties"))
        if p is None:  # a sandbox may hide other jobs' GPUs (EPERM); ROCr skips them too
            _UNREADABLE += 1
            continue
        if not p.get("gfx_target_version"):
            continue
        loc, dom = p.get("location_id", 0), p.get("domain", 0)
        bdf = "%04x:%02x:%02x.%x" % (dom, (loc >> 8) & 0xFF, (loc >> 3) & 0x1F, loc & 0x7)
        gpus.append({"node": i, "gfx_target_version": p["gfx_target_version"], "bdf": bdf,
                     "unique_id": p.get("unique_id", 0)})
    return gpus


def _filter(devs, spec):
    """Apply one *_VISIBLE_DEVICES value: comma-separated indices or GPU-<hex> UUIDs; as in
    the runtimes, the list ends at the first entry that names no device."""
    if spec is None:
        return devs
    out = []
    for tok in spec.split(","):
        tok = tok.strip()
        if not tok:
            break
        pick = None
        if tok.isdigit():
            i = int(tok)
            pick = devs[i] if i < len(devs) else None
        elif tok.upper().startswith("GPU-"):
            want = tok[4:].lower()
            pick = next((d for d in devs if "%x" % d.get("unique_id", 0) == want.lstrip("0") or
                         "%016x" % d.get("unique_id", 0) == want), None)
        if pick is None or pick in out:
            break
        out.append(pick)
    return out


def visible_gpus(env=None, sysfs=None):
    """The GPUs HIP will number 0..n-1 in a process started with `env`, or None if unknown."""
    sysfs = SYSFS if sysfs is None else sysfs
    env = os.environ if env is None else env
    devs = kfd_gpus(sysfs)
    if devs is None:
        return None
    devs = _filter(devs, env.get("ROCR_VISIBLE_DEVICES"))
    # HIP reads HIP_VISIBLE_DEVICES, else CUDA_VISIBLE_DEVICES; an empty value is its default,
    # i.e. no filter (this build container exports HIP_VISIBLE_DEVICES= )
    hip = env.get("HIP_VISIBLE_DEVICES") or env.get("CUDA_VISIBLE_DEVICES") or None
    devs = _filter(devs, hip)
    return devs


def gpu_count(env=None, sysfs=None):
    """(count, source) without any HIP call.  count is None when sysfs does not say for sure:
    the topology is unreadable, or some of its nodes are (then the count is only a lower
    bound, and the launcher leaves the check to the ranks)."""
    sysfs = SYSFS if sysfs is None else sysfs
    devs = visible_gpus(env, sysfs)
    if devs is None:
        return None, "kfd topology unreadable"
    src = "kfd topology (%s)" % os.path.join(sysfs, KFD_NODES)
    if _UNREADABLE:
        return None, "%s: %d readable GPU node(s), %d node(s) unreadable" % (src, len(devs), _UNREADABLE)
    return len(devs), src


def bdf_of_torch_device(props):
    """The PCI function of a torch device-properties object (pci_domain_id/bus_id/device_id), or None."""
    try:
        return "%04x:%02x:%02x.0" % (props.pci_domain_id, props.pci_bus_id, props.pci_device_id)
    except (AttributeError, TypeError):
        return None


def bind_bdf(bdf, sysfs=None, apply=True):
    """Bind to the NUMA node of the PCI function `bdf` (the rank's post-init check)."""
    sysfs = SYSFS if sysfs is None else sysfs
    base = os.path.join(sysfs, PCI_DEVICES, bdf)
    node_txt = _read(os.path.join(base, "numa_node"))
    node = int(node_txt) if node_txt and node_txt.strip().lstrip("-").isdigit() else -1
    cpus = parse_cpulist(_read(os.path.join(base, "local_cpulist")))
    rec = {"bdf": bdf, "numa_node": node, "bound": False}
    mine = os.sched_getaffinity(0)
    target = cpus & mine
    if target and apply:
        os.sched_setaffinity(0, target)
        rec.update(bound=True, cpus=len(target))
    return rec


def gpu_numa(local, env=None, sysfs=None):
    """NUMA placement of HIP device `local`: {'bdf', 'numa_node', 'cpus'} (cpus a set), or None."""
    sysfs = SYSFS if sysfs is None else sysfs
    devs = visible_gpus(env, sysfs)
    if not devs or not 0 <= local < len(devs):
        return None
    bdf = devs[local]["bdf"]
    base = os.path.join(sysfs, PCI_DEVICES, bdf)
    node_txt = _read(os.path.join(base, "numa_node"))
    node = int(node_txt) if node_txt and node_txt.strip().lstrip("-").isdigit() else -1
    cpus = parse_cpulist(_read(os.path.join(base, "local_cpulist")))
    if not cpus and node >= 0:
        cpus = parse_cpulist(_read(os.path.join(sysfs, "sys/devices/system/node", "node%d" % node, "cpulist")))
    return {"bdf": bdf, "numa_node": node, "cpus": cpus, "kfd_node": devs[local]["node"]}


def bind_rank(local, env=None, sysfs=None, apply=True):
    """Restrict this thread (and every thread it starts later) to the CPUs of GPU `local`'s
    NUMA node that it may run on.  Returns the record bench.py puts in its line."""
    sysfs = SYSFS if sysfs is None else sysfs
    rec = {"local_rank": local, "numa_node": None, "bdf": None, "bound": False, "cpus": None}
    try:
        mine = os.sched_getaffinity(0)
    except (AttributeError, OSError):
        rec["reason"] = "no sched_getaffinity"
        return rec
    place = gpu_numa(local, env, sysfs)
    if place is None:
        rec["reason"] = "GPU placement unknown (kfd topology unreadable or index out of range)"
        rec["cpus"] = len(mine)
        return rec
    rec.update(bdf=place["bdf"], numa_node=place["numa_node"])
    target = place["cpus"] & mine
    if not place["cpus"]:
        rec["reason"] = "device reports no local CPUs"
    elif not target:
        rec["reason"] = "none of the node's CPUs is in this process's affinity mask"
    elif target == mine:
        rec.update(bound=True, reason="affinity already within the node")
    elif apply:
        os.sched_setaffinity(0, target)
        rec.update(bound=True, reason="bound to the node's CPUs")
    else:
        rec.update(bound=True, reason="would bind (dry run)")
    rec["cpus"] = len(target) if rec["bound"] else len(mine)
    return rec


def cgroup_cpu_quota(sysfs=None):
    """CPUs allowed by the cgroup CPU quota (v2 cpu.max or v1 cfs_quota/period), or None."""
    sysfs = SYSFS if sysfs is None else sysfs
    v2 = _read(os.path.join(sysfs, "sys/fs/cgroup/cpu.max"))
    if v2:
        q, _, p = v2.strip().partition(" ")
        if q != "max" and q.isdigit() and p.isdigit() and int(p) > 0:
            return int(q) / int(p)
        return None
    q = _read(os.path.join(sysfs, "sys/fs/cgroup/cpu/cpu.cfs_quota_us"))
    p = _read(os.path.join(sysfs, "sys/fs/cgroup/cpu/cpu.cfs_period_us"))
    try:
        q, p = int(q), int(p)
    except (TypeError, ValueError):
        return None
    return q / p if q > 0 and p > 0 else None


def cpu_share(sysfs=None):
    """What this process may actually run on: the machine's CPU count, its affinity mask and
    the cgroup quota; `usable` is the smallest of them (whole CPUs)."""
    sysfs = SYSFS if sysfs is None else sysfs
    visible = os.cpu_count()
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = visible
    quota = cgroup_cpu_quota(sysfs)
    usable = aff if quota is None else max(1, min(aff, int(quota)))
    return {"nproc": visible, "affinity": aff, "cgroup_quota_cpus": quota, "usable": usable}


def open_gpu_fds(pid="self"):
    """Paths of this process's open fds that are GPU device nodes (/dev/kfd, /dev/dri/*)."""
    out = []
    d = "/proc/%s/fd" % pid
    try:
        names = os.listdir(d)
    except OSError:
        return out
    for fd in names:
        try:
            tgt = os.readlink(os.path.join(d, fd))
        except OSError:
            continue
        if tgt == "/dev/kfd" or tgt.startswith("/dev/dri/"):
            out.append(tgt)
    return out
