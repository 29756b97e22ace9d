#!/usr/bin/env python3
"""Benchmark: Lanczos iterations/s and achieved SpMV HBM GB/s on the 3-D Poisson 7-point matrix,
256^3 DoF (BASELINE.json metric), fp64, 1..8 MI355X.

One "step" = one Lanczos three-term-recurrence iteration (no re-orthogonalisation) of the whole
256^3 problem: by default the fused one-reduction step (one kernel: t = A u sig - gam u_prev and the
step's three sums), plus at N > 1 the one-plane RCCL halo exchange and one 3-value
allreduce.  The matrix is row-partitioned in z-slabs (strong scaling: the total work is fixed as N
grows).

The timed image reads every stored matrix value from HBM on every step, as BCRSMatrix::mv does
(kernels_cpp.hh:611-617): `--image arrays` (default) = the symmetric band arrays (EIG_MAT_NO_UNIFORM:
the 4 upper diagonals, 32 B per row, lower entries through the mirrored slots).  At N = 1 the line
also carries the same step on the SELL / CSR image (`csr`: values + column structure) and the
constant-coefficient shortcut (`stencil_shortcut`: band values in the kernel arguments, no matrix
bytes) -- side numbers, never `value` or `roofline`.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
        bench.py --gpus N --steps K --warmup W

`--gpus N` (N > 1) without a launcher (WORLD_SIZE unset) starts the N ranks itself: a
torch.distributed.run child with --nproc-per-node N, launched before this process touches the GPU
(libeigmi is imported only after that decision); its one JSON line is forwarded, and a line whose
n_gpus or comm.nranks differs from N fails the run.  Under a launcher, WORLD_SIZE must equal --gpus.

torch.distributed (gloo) is only the bootstrap / barrier / max-over-ranks channel; the data path
is libeigmi's own RCCL communicator over xGMI.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd"))

import numpy as np  # noqa: E402

eigmi = None  # libeigmi (loads the HIP library): imported by load_eigmi() once the launch is decided


def load_eigmi():
    global eigmi
    if eigmi is None:
        import eigmi as _e
        eigmi = _e
    return eigmi


# ----------------------------------------------------------------------------- N-rank launcher
def launcher_command(gpus, argv, port):
    """The torch.distributed.run command that runs this script on `gpus` ranks of this node."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def child_line(text, gpus):
    """The N-rank child's stdout -> (its JSON line as a dict or None, error or None): exactly one
    JSON line, n_gpus == gpus and comm.nranks == gpus (RCCL saw every rank)."""
    lines = [ln for ln in text.splitlines() if ln.lstrip().startswith("{")]
    if len(lines) != 1:
        return None, f"expected one JSON line from the {gpus}-rank run, got {len(lines)}"
    try:
        d = json.loads(lines[0])
    except ValueError as e:
        return None, f"unparsable line from the {gpus}-rank run: {e}"
    if d.get("n_gpus") != gpus:
        return d, f"the {gpus}-rank run reported n_gpus = {d.get('n_gpus')}"
    nr = (d.get("comm") or {}).get("nranks")
    if nr != gpus:
        return d, f"the {gpus}-rank run's communicator has {nr} ranks"
    return d, None


def run_ranks(gpus, argv):
    """Run this script on `gpus` ranks (child launcher; nothing here has touched the GPU) and forward
    its JSON line; the exit status is the child's, or 4 when its line does not show `gpus` ranks."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL across processes)
    cmd = launcher_command(gpus, argv, free_port())
    print("bench: " + " ".join(cmd), file=sys.stderr, flush=True)
    p = subprocess.run(cmd, stdout=subprocess.PIPE, env=env)
    d, err = child_line(p.stdout.decode(errors="replace"), gpus)
    if p.returncode != 0:
        print(f"bench: the {gpus}-rank run failed with status {p.returncode}", file=sys.stderr)
        return p.returncode
    if err:
        print("bench: " + err, file=sys.stderr)
        return 4
    sys.stdout.write(json.dumps(d) + "\n")
    sys.stdout.flush()
    return 0


def world_from_env(gpus):
    """(world, rank, local rank) under a launcher; --gpus must match WORLD_SIZE (None: take it)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if gpus is not None and gpus != world:
        raise SystemExit(f"bench: --gpus {gpus} but WORLD_SIZE={world}")
    return world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def ab_mismatch(a1, b1, a2, b2):
    """Largest relative difference of two Lanczos coefficient sequences over their common steps."""
    k = min(len(a1), len(a2))
    if k == 0:
        return 0.0
    ra = np.abs(np.asarray(a1[:k]) - np.asarray(a2[:k])) / np.maximum(np.abs(np.asarray(a2[:k])), 1e-300)
    kb = min(len(b1), len(b2))
    rb = np.abs(np.asarray(b1[:kb]) - np.asarray(b2[:kb])) / np.maximum(np.abs(np.asarray(b2[:kb])), 1e-300)
    m = max(float(ra.max()), float(rb.max()) if kb else 0.0)
    return m if np.isfinite(m) else float("inf")


AB_RTOL = 1e-12  # a non-RCCL transport must reproduce the RCCL run's alpha / beta to this

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def cpu_baseline(N, rp, c, v, steps, gpu_alpha, fused):
    """The Lanczos step on the CPU (oracle restatement: a3 SpMV + the BLAS-1 loops of ARPACK; the
    same variant the GPU ran), single thread, same matrix and start vector; a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # noqa: E402  (checker / baseline only)
    n = N ** 3
    u0, u1, u2 = np.zeros(n), np.zeros(n), np.zeros(n)
    oracle.lib.orc_random_vec(n, 123, u0)
    alpha, beta = np.zeros(steps), np.zeros(steps + 1)
    fast = oracle.fast_lib()  # -O3 -march=x86-64-v3 build of the restatement (oracle/Makefile)
    t0 = time.perf_counter()
    if fused:
        fast.orc_lanczos_fused(n, rp, c, v, steps, u0, alpha, beta, None)
    else:
        fast.orc_lanczos_rotating(n, rp, c, v, steps, u0, u1, u2, alpha, beta)
    dt = time.perf_counter() - t0
    k = min(steps, len(gpu_alpha))
    rel = float(np.max(np.abs(alpha[:k] - gpu_alpha[:k]) / np.abs(alpha[:k]))) if k else None
    return steps / dt, dt, rel


def scipy_crosscheck(N, rp, c, v, steps, gpu_alpha):
    """Same-host cross-check of the CPU baseline with a third-party implementation: the plain Lanczos
    recurrence (w = A v - beta v_prev; alpha = w.v; w -= alpha v; beta = ||w||) on scipy.sparse's CSR
    matvec (ARPACK's operator in scipy.sparse.linalg.eigsh) and numpy BLAS-1, single thread, same
    matrix and start vector as the oracle baseline; a bounded sample of `steps` steps."""
    import scipy.sparse as sp
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # noqa: E402  (the start vector generator only)
    n = N ** 3
    A = sp.csr_matrix((v, c, rp), shape=(n, n), copy=False)
    q = np.zeros(n)
    oracle.lib.orc_random_vec(n, 123, q)
    q /= np.linalg.norm(q)
    qprev, beta = np.zeros(n), 0.0
    alpha = np.zeros(steps)
    t0 = time.perf_counter()
    for j in range(steps):
        w = A @ q
        w -= beta * qprev
        alpha[j] = w @ q
        w -= alpha[j] * q
        beta = float(np.linalg.norm(w))
        qprev, q = q, w / beta
    dt = time.perf_counter() - t0
    k = min(steps, len(gpu_alpha))
    rel = float(np.max(np.abs(alpha[:k] - gpu_alpha[:k]) / np.abs(alpha[:k]))) if k else None
    return steps / dt, dt, rel


def cpu_replicas(N, rp0, c0, v0, steps, fused, threads):
    """SURVEY 8(d) CPU baseline (ii): the reference's own parallel mode (src/dune-eigensolver.cc:
    754-760, aggregate as at :292-294) -- `threads` independent replicas of the single-thread solve,
    each on its own copy of the matrix (rp0, c0, v0) and vectors, started together behind a barrier;
    value = replicas x steps / wall time.  ctypes drops the GIL, so the replicas run in parallel."""
    import threading
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # noqa: E402  (checker / baseline only)
    n = N ** 3
    bar = threading.Barrier(threads + 1)
    err = []

    def replica():
        try:
            rp, c, v = rp0.copy(), c0.copy(), v0.copy()
            u0, u1, u2 = np.zeros(n), np.zeros(n), np.zeros(n)
            oracle.lib.orc_random_vec(n, 123, u0)
            alpha, beta = np.zeros(steps), np.zeros(steps + 1)
        except MemoryError as e:  # pragma: no cover
            err.append(e)
        bar.wait()  # all replicas built
        bar.wait()  # go
        if not err:
            fast = oracle.fast_lib()
            if fused:
                fast.orc_lanczos_fused(n, rp, c, v, steps, u0, alpha, beta, None)
            else:
                fast.orc_lanczos_rotating(n, rp, c, v, steps, u0, u1, u2, alpha, beta)
        bar.wait()  # done

    ts = [threading.Thread(target=replica) for _ in range(threads)]
    for t in ts:
        t.start()
    bar.wait()
    t0 = time.perf_counter()
    bar.wait()
    bar.wait()
    dt = time.perf_counter() - t0
    for t in ts:
        t.join()
    if err:
        return None, dt
    return threads * steps / dt, dt


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def committed_traffic(kernel, N, world, build, image):
    """HBM bytes per launch of `kernel` (a template instance "k_...<...>" matches exactly, a bare name
    any instance) from the committed rocprofv3 PMC summaries (profiles/<tag>_pmc_summary.json,
    FETCH_SIZE x2 + WRITE_SIZE, KiB -> B; tools/profile_round.sh) taken on the same configuration and
    matrix image: the newest one profiled on this build (eigmi.build_id()) when there is one, else the
    newest of any build; (bytes, source, same_build) or None."""
    import glob
    best = None
    for p in glob.glob(os.path.join(ROOT, "profiles", "*_pmc_summary.json")):
        try:
            d = json.load(open(p))
            line = d.get("bench_line_under_trace")
            cfg = line.get("config") if isinstance(line, dict) else None
            if not isinstance(cfg, dict) or cfg.get("N") != N or line.get("n_gpus") != world:
                continue
            if cfg.get("image", "uniform") != image:
                continue
            for name, k in d["kernels"].items():  # template instances: "eigmi::k_..._b1<1, 1>"
                if (name == "eigmi::" + kernel) if "<" in kernel else (name.split("<")[0] == "eigmi::" + kernel):
                    same = d.get("build") is not None and d.get("build") == build
                    stamp = (same, d.get("collected", os.path.getmtime(p)))
                    if best is None or stamp > best[2]:
                        best = (k["hbm_bytes"], os.path.relpath(p, ROOT), stamp)
        except (OSError, ValueError, KeyError, TypeError, AttributeError):
            continue
    return (best[0], best[1], best[2][0]) if best else None


def comm_summary(ctx, world, ab_check):
    ci = ctx.comm_info()
    cc = ctx.comm_counters()
    return {"nranks": ci["nranks"], "allreduce": ci["allreduce"],
            "mailbox_errors": ci["mailbox_errors"], "allreduce_calls": cc["allreduce"] + cc["allreduce_split"],
            "halo_groups": cc["halo_groups"], "transport_check": ab_check or None}


MAILBOX_KINDS = ("xgmi-mailbox", "xgmi-mailbox-step")  # eig_comm_info: a validated mailbox in use

VARIANT_NAME = {"fused": "fused one-reduction step", "pipelined": "pipelined one-reduction step",
                "classic": "SpMV + update kernels"}
# matrix images (eig_mat_create_bcsr_ex flags)
IMAGES = ("arrays", "csr", "uniform")


def image_flags(image):
    return {"arrays": eigmi.MAT_NO_UNIFORM, "csr": eigmi.MAT_NO_BAND, "uniform": 0}[image]


def image_name(M):
    """What the step kernel streams on this image (config.matrix_image)."""
    info = M.info
    v = info.march_variant
    if info.sym_offsets == 0:
        return "SELL-64 / CSR image (values + column structure: stencil slices keep offsets + a 1-B row mask)"
    if v == 15:
        return ("symmetric band values streamed every step as two pair arrays ((+D, 0) and (+1, +nx) per row: "
                "the 4 upper diagonals, 32 B per row; lower entries through the mirrored slots; row masks from "
                "the grid coordinates; the (t, u) pairs streamed)")
    if v >= 10:
        return (f"symmetric band arrays streamed every step ({info.sym_arrays} upper diagonals, "
                f"{8 * info.sym_arrays} B per row; lower entries through the mirrored slots; row masks from "
                f"the grid coordinates; the (t, u) pairs streamed)")
    if v >= 2:
        return ("uniform band on a grid (constant coefficients: the band values in the kernel arguments, row "
                "masks from the grid coordinates; the (t, u) pairs streamed -- reads no matrix bytes)")
    if v == 1:
        return "uniform band (band values in the kernel arguments, 1-B row mask + (t, u) pairs streamed)"
    return "symmetric band arrays + 1-B row mask streamed every step"


def kernel_instance(M, kname):
    """The template instance of a march or SELL-slice kernel (as rocprofv3 names it), else the bare
    name.  SELL slice kernels: <R = 1, image mode> (k_spmv.hip: 0 explicit columns, 1 all slices
    stencil, 2 mixed)."""
    info = M.info
    if kname.endswith("_march") and info.march_variant >= 0 and info.sym_mask_bytes == 1 and info.sym_offsets <= 7:
        return f"{kname}<unsigned char, true, {info.march_variant}>"
    if kname.endswith("_b1") and info.sym_offsets == 0:
        mode = 0 if info.stencil_slices == 0 else 1 if info.stencil_slices == info.nslices else 2
        if kname in ("k_lanczos_fused_b1", "k_spmv_b1"):
            # <R, mode, CPF>: the explicit slices' column prefetch is a measurement switch (eigmi.h
            # EIG_TUNE_SELL_CPF), off in the bench
            cpf = False
            return f"{kname}<1, {mode}, {'true' if cpf else 'false'}>"
        return f"{kname}<1, {mode}>"
    return kname


def side_image(ctx, rp, c, v, image, steps, n, nnz, traffic=None, flags=None, extra=None):
    """N = 1 side measurement: the same fused step on another image of the same matrix (K eager steps,
    region events: one launch per step), priced at the bytes that image streams (the kernel's byte
    model: eig_lanczos_kernel_info -- for the SELL-64 image its padded values, column indices of the
    explicit slices, stencil offsets and row masks, not the CSR count) with the committed PMC traffic
    of the same kernel beside it, and at SURVEY 8(d)'s CSR step bytes."""
    M = eigmi.Matrix.from_bcsr(ctx, rp, c, v, flags=image_flags(image) if flags is None else flags)
    try:
        ws = eigmi.LanczosWorkspace(M, steps + 5, seed=123, fused=True)
        ws.step(5)
        ctx.sync()
        t0 = time.perf_counter()
        tim = ws.step(steps)
        ctx.sync()
        dt = time.perf_counter() - t0
        kname, kb = M.lanczos_kernel_info(True)
        ws.close()
        us = tim.total_ms / steps * 1e3
        sb = eigmi.bytes_lanczos_step(n, nnz)
        ki = kernel_instance(M, kname)
        out = {"image": image, "matrix_image": image_name(M), "kernel": ki,
               "value": round(steps / dt, 3), "unit": "iters/s", "ms_per_step": round(dt / steps * 1e3, 4),
               "avg_launch_us": round(us, 2), "bytes_per_launch": kb,
               "achieved_GBs": round(kb / us / 1e3, 1), "frac": round(kb / us / 1e3 / HBM_PEAK_GBS, 4),
               "survey_step_bytes": sb, "survey_step_GBs": round(sb / (dt / steps) / 1e9, 1),
               "survey_step_frac": round(sb / (dt / steps) / 1e9 / HBM_PEAK_GBS, 4)}
        tr = traffic(ki) if traffic else None
        if tr:
            out.update({"traffic": tr[0], "traffic_source": tr[1], "traffic_same_build": tr[2],
                        "traffic_vs_bytes": round(tr[0] / kb, 4),
                        "traffic_frac": round(tr[0] / us / 1e3 / HBM_PEAK_GBS, 4)})
        if extra:
            out.update(extra)
        return out
    finally:
        M.close()


def side_general(ctx, N, steps, traffic, seed=123):
    """N = 1 side measurement on a GENERAL sparse matrix: the same 3-D Poisson N^3 under a seeded
    random symmetric permutation and reverse Cuthill-McKee (eigmi.scrambled_rcm, tools/csr_general.py):
    same nnz, no constant-offset band, explicit column indices in most SELL slices -- what an
    unstructured BCRSMatrix looks like to the kernels.  Reordering on the host is outside the timing."""
    t0 = time.perf_counter()
    rp, c, v = eigmi.gen_matrix(eigmi.GEN_POISSON3D, N)
    rp, c, v = eigmi.scrambled_rcm(rp, c, v, seed)
    t_re = time.perf_counter() - t0
    n, nnz = rp.size - 1, int(rp[-1])
    rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(rp))
    bw = int(np.abs(c - rows).max())
    del rows
    return side_image(ctx, rp, c, v, "csr", steps, n, nnz, traffic=traffic, flags=0,
                      extra={"matrix": f"3-D Poisson {N}^3 scrambled (seed {seed}) + RCM: bandwidth {bw}",
                             "reorder_s": round(t_re, 1)})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); N > 1 without a launcher starts torch.distributed.run itself")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--N", type=int, default=256, help="grid points per axis (n = N^3)")
    ap.add_argument("--matrix", choices=["poisson", "varcoef"], default="poisson",
                    help="poisson: the 7-point Poisson matrix of the metric (eig_gen kind 4); varcoef: the "
                         "same pattern with a hashed conductance per grid edge (kind 8)")
    ap.add_argument("--image", choices=list(IMAGES), default="arrays",
                    help="matrix image of the timed step: arrays = symmetric band arrays streamed every step "
                         "(EIG_MAT_NO_UNIFORM), csr = SELL / CSR image (EIG_MAT_NO_BAND), uniform = the "
                         "constant-coefficient shortcut (band values in the kernel arguments, no matrix bytes)")
    ap.add_argument("--side-steps", type=int, default=50,
                    help="N = 1: steps of the csr / stencil_shortcut side measurements (0 = skip them)")
    ap.add_argument("--general-steps", type=int, default=30,
                    help="N = 1: steps of the general-matrix side measurement (scrambled + RCM; 0 = skip)")
    ap.add_argument("--cpu-steps", type=int, default=160, help="Lanczos steps of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-replicas", type=int, default=None,
                    help="replicas of the CPU baseline's parallel mode (default: usable cores, at most 16; 0 = skip)")
    ap.add_argument("--cpu-replica-steps", type=int, default=40)
    ap.add_argument("--scipy-steps", type=int, default=20, help="steps of the scipy.sparse cross-check sample")
    ap.add_argument("--no-kernel-events", action="store_true", help="skip per-kernel HIP events")
    ap.add_argument("--kernel-events", choices=["auto", "per-launch"], default="auto",
                    help="auto: region events at N=1 for the fused step, per-launch events otherwise")
    ap.add_argument("--variant", choices=["auto", "fused", "pipelined", "classic"], default="auto",
                    help="fused: one kernel + one 3-value allreduce per step (EIG_LANCZOS_FUSED); "
                         "pipelined: SpMV on t_{k-1} overlapping the previous step's allreduce + a row "
                         "kernel (EIG_LANCZOS_PIPELINED); classic: SpMV kernel + update kernel, two "
                         "allreduces; auto: fused on one GPU, on N > 1 the faster of fused / pipelined "
                         "in a short timed trial before the timed region (all ranks agree)")
    ap.add_argument("--trial-steps", type=int, default=40, help="steps per variant of the auto trial (N > 1)")
    ap.add_argument("--rehearse-trial", action="store_true",
                    help="run the N > 1 auto trial (variant x launch) on one GPU too (rehearsal of that path)")
    ap.add_argument("--comm-self", action="store_true",
                    help="one GPU: attach a one-rank RCCL communicator with EIG_COMM_ALWAYS, so every step's "
                         "allreduce runs through ncclAllReduce (the transport's per-step cost without xGMI)")
    ap.add_argument("--allreduce", choices=["auto", "rccl", "mailbox", "mailbox-step"], default="auto",
                    help="N > 1: the step's allreduce transport -- ncclAllReduce, the xGMI mailbox (one "
                         "launch stores the 3 sums into every peer's mailbox; set up and validated by all "
                         "ranks, else RCCL), or mailbox-step (the fused step's sums published by its last "
                         "workgroup and gathered in the next launch's prologue: no allreduce launch); auto = "
                         "all in the trial, the fastest whose alpha / beta match the RCCL run wins")
    ap.add_argument("--transport", choices=["rccl", "mailbox-only"], default="rccl",
                    help="N > 1: rccl = libeigmi's RCCL communicator (+ the mailbox unless --allreduce rccl); "
                         "mailbox-only = no RCCL, every exchange over the xGMI mailbox (eig_comm_ipc_open: the "
                         "handles travel over gloo) -- with EIGMI_FORCE_DEVICE=0 the whole N-rank run rehearsed "
                         "on ONE GPU, which RCCL refuses")
    ap.add_argument("--launch", choices=["auto", "graph", "eager"], default="auto",
                    help="timed steps as one hipGraph replay or launched one by one; auto = graph when "
                         "N > 1 (host-bound halo/allreduce calls), eager at N = 1 (measured faster there)")
    args = ap.parse_args()
    if args.gpus is not None and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # decided before anything loads the HIP library or touches the GPU
        sys.exit(run_ranks(args.gpus, sys.argv[1:]))
    world, rank, local = world_from_env(args.gpus)
    load_eigmi()
    # stdout carries exactly one JSON line: native libraries that write to fd 1 (RCCL prints its
    # version banner there at communicator creation) are sent to stderr, the line goes to the saved fd
    sys.stdout.flush()
    out_fd = os.dup(1)
    os.dup2(2, 1)

    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")

    def barrier():
        if dist is not None:
            dist.barrier()

    # EIGMI_FORCE_DEVICE pins every rank to one device: it rehearses only the bootstrap (RCCL 2.27
    # refuses two ranks on one device with ncclInvalidUsage at ncclCommInitRank, profiles/r04t_*)
    ctx = eigmi.Context(int(os.environ.get("EIGMI_FORCE_DEVICE", local)))
    if world == 1 and args.comm_self:
        # one-rank RCCL communicator (+ the mailbox unless --allreduce rccl): the transports' per-step
        # cost on one GPU
        ctx.comm_init(1, 0, eigmi.Context.unique_id(), mailbox=args.allreduce != "rccl", always=True)
        if args.allreduce not in ("auto",):
            ctx.select_allreduce(args.allreduce)
        elif not args.rehearse_trial:
            ctx.select_allreduce("rccl")
    if world > 1:
        import torch
        uid = eigmi.Context.unique_id() if rank == 0 else bytes(128)
        t = torch.tensor(list(uid), dtype=torch.uint8)
        dist.broadcast(t, 0)
        if args.transport == "mailbox-only":
            # every rank's mailbox handle to every rank over gloo, then all open them
            h = torch.tensor(list(ctx.ipc_handle(world, rank)), dtype=torch.uint8)
            hs = [torch.zeros_like(h) for _ in range(world)]
            dist.all_gather(hs, h)
            ctx.ipc_open(b"".join(bytes(x.tolist()) for x in hs))
        else:
            # RCCL, plus the xGMI mailbox allreduce where every rank validates it (eig_comm_init_ex
            # EIG_COMM_MAILBOX; agreed by all ranks, else RCCL alone) -- the auto trial times both
            ctx.comm_init(world, rank, bytes(t.tolist()), mailbox=args.allreduce != "rccl")
    mb_only = world > 1 and args.transport == "mailbox-only"

    N = args.N
    n = N ** 3
    b, cnt = eigmi.row_partition(n, world, rank, align=N * N)
    gkind = eigmi.GEN_VARCOEF3D if args.matrix == "varcoef" else eigmi.GEN_POISSON3D
    rp, c, v = eigmi.gen_rows(gkind, N, b, cnt)
    if world > 1:
        M = eigmi.Matrix.from_rows(ctx, n, b, rp, c, v, flags=image_flags(args.image))
    else:
        M = eigmi.Matrix.from_bcsr(ctx, rp, c, v, flags=image_flags(args.image))
    nnz_total = int(eigmi.lib.eig_gen_nnzb(gkind, N))
    nnz_local = int(rp[-1])

    K, W = args.steps, args.warmup
    build = eigmi.build_id()

    def max_over_ranks(x):
        if dist is None:
            return x
        import torch
        tt = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item())

    # N > 1: the per-step allreduce sits on the fused step's critical path; the pipelined step hides
    # it behind the next SpMV at 56 B/row of extra row traffic.  Which wins depends on the
    # allreduce latency over xGMI, so the auto variant measures both (graph replays, max over ranks)
    variant = args.variant
    trial = None
    ab, ab_check = {}, {}
    halo_mode = "split"
    halo_x = "rccl"
    if variant == "auto":
        # one rank: EIG_LANCZOS_AUTO's choice for this image (the fused step on a 1x1 image)
        tw = eigmi.LanczosWorkspace(M, 1, seed=123, fused="auto")
        variant = tw.variant
        tw.close()
        if world > 1 or args.rehearse_trial:
            trial = {}
            # halo: "split" = interior planes during the exchange + a boundary launch (the default),
            # "whole" = the exchange first, then one launch (EIG_TUNE_HALO; no second launch's fixed
            # cost) -- N > 1 only, one GPU has no halo
            halos = ("split", "whole") if world > 1 else ("split",)
            multi = world > 1 or args.comm_self
            have_mb = multi and ctx.comm_info()["allreduce"] in MAILBOX_KINDS
            ars = ((("rccl", "mailbox", "mailbox-step") if args.allreduce == "auto" else (args.allreduce,))
                   if have_mb else ("rccl",))
            if mb_only:
                ars = ("mailbox", "mailbox-step")  # mailbox-only ranks: the allreduce launch is the reference
            ref_ar = "mailbox" if mb_only else "rccl"
            if ref_ar not in ars:
                ars = (ref_ar,) + ars  # the reference run of the alpha / beta check
            # (the pipelined step keeps the allreduce launch under mailbox-step: same as mailbox)
            # N > 1 with the mailbox: the halo also through the halo mailbox (eig_comm_select_halo; the
            # boundary planes stored into the peers' staging over xGMI) beside ncclSend / ncclRecv
            # (--rehearse-trial: selected at one rank too, where no matrix has a halo)
            hx_ok = (world > 1 or args.rehearse_trial) and have_mb and not mb_only
            hxs_mb = ("rccl", "mailbox") if hx_ok else ("rccl",)
            if len(hxs_mb) > 1:
                # the halo mailbox's staging is built at matrix creation; a rank set that could not build
                # it (agreed there) keeps ncclSend / ncclRecv, and every rank gets the same answer here
                try:
                    ctx.select_halo("mailbox")
                    ctx.select_halo("rccl")
                except eigmi.EigError as e:
                    print(f"bench: halo mailbox unavailable ({e}); RCCL halo only", file=sys.stderr, flush=True)
                    hxs_mb = ("rccl",)
            combos = [(v, h, a, x) for v in ("fused", "pipelined") for h in halos for a in ars
                      for x in (hxs_mb if a != "rccl" else ("rccl",))
                      if not (v == "pipelined" and a == "mailbox-step")]
            for var, halo, ar, hx in combos:
                M.tune(halo_whole=int(halo == "whole"))
                if multi:
                    ctx.select_allreduce(ar)
                if len(hxs_mb) > 1:
                    ctx.select_halo(hx)
                tkey = f"{halo}/{ar}" + ("/halo-mailbox" if hx == "mailbox" else "")
                # every call below may already have queued a halo exchange or an allreduce on the
                # other ranks when it fails here, so a failing rank cannot rejoin them at a barrier:
                # it exits non-zero at once and the launcher tears the job down on every rank
                # (a refused hipGraph capture is no failure: replay() then runs the steps eagerly)
                # --launch auto also times the eager loop: a hipGraph replay adds a few us per kernel
                # node on this stack (one GPU, 128^3 fused step: 22.2 us per step replayed vs 18.3
                # eager, profiles/r03bx_*), which can outweigh the host's per-step enqueue cost
                launches = ("graph", "eager") if args.launch == "auto" else (args.launch,)
                tw = None
                ms = {}
                try:
                    tw = eigmi.LanczosWorkspace(M, 5 + len(launches) * args.trial_steps, seed=123,
                                                fused=var == "fused", pipelined=var == "pipelined")
                    tw.step(5)
                    for la in launches:
                        if la == "graph":
                            tw.capture(args.trial_steps)
                        barrier()
                        ctx.sync()
                        t0 = time.perf_counter()
                        if la == "graph":
                            tw.replay()
                        else:
                            tw.step(args.trial_steps)
                        ctx.sync()
                        ms[la] = (time.perf_counter() - t0) / args.trial_steps * 1e3
                    ab[(var, halo, ar, hx)] = tw.tridiag()
                except eigmi.EigError as e:
                    if not (ar == "mailbox-step" and e.code == eigmi.EIG_ERR_RCCL):
                        print(f"bench: {var} trial failed on rank {rank}: {e}; stopping every rank", file=sys.stderr,
                              flush=True)
                        os._exit(3)
                    # a timed-out in-kernel exchange: every rank reads NaN sums and stops at the same
                    # launch (csrc/xch_dev.h), so the ranks stay in step -- the transport is out
                    print(f"bench: {var} trial on {ar}: {e}", file=sys.stderr, flush=True)
                    ms = {la: float("inf") for la in launches}
                finally:
                    if tw is not None:
                        tw.close()
                barrier()
                # a mailbox call that timed out on some rank (its sums read NaN): not a candidate
                # (checked per combination: selecting a transport clears the recorded timeouts)
                failed = ar != "rccl" and max_over_ranks(ctx.comm_info()["mailbox_errors"]) > 0
                for la in launches:
                    trial[f"{var}/{la}/{tkey}"] = float("inf") if failed else round(max_over_ranks(ms[la]), 4)
            # a transport is a candidate only if its run reproduces the RCCL run of the same variant
            # and halo mode (same start vector, same step count) to AB_RTOL -- never on timing alone
            for (var, halo, ar, hx), (a, b) in ab.items():
                if ar == ref_ar and hx == "rccl":
                    continue
                ref = ab.get((var, halo, ref_ar, "rccl"))
                mm = ab_mismatch(a, b, *ref) if ref is not None else float("inf")
                mm = max_over_ranks(mm)
                ok = mm <= AB_RTOL
                tkey = f"{halo}/{ar}" + ("/halo-mailbox" if hx == "mailbox" else "")
                ab_check[f"{var}/{tkey}"] = {"max_rel_diff_vs_rccl": mm if np.isfinite(mm) else None,
                                             "reference": ref_ar, "steps": int(len(a)), "ok": bool(ok)}
                if not ok:
                    for k in trial:
                        if k.startswith(f"{var}/") and k.split("/", 2)[2] == tkey:
                            trial[k] = float("inf")
            best = min(trial, key=trial.get)
            parts = best.split("/")
            variant, best_launch, best_halo, best_ar = parts[:4]
            if args.launch == "auto":
                args.launch = best_launch
            M.tune(halo_whole=int(best_halo == "whole"))
            if multi:
                ctx.select_allreduce(best_ar)
            halo_x = "mailbox" if len(parts) > 4 or mb_only else "rccl"
            if len(hxs_mb) > 1:
                ctx.select_halo(halo_x)
            halo_mode = best_halo
    if world > 1 and trial is None:
        # no trial: RCCL unless a mailbox transport was asked for (and is set up on every rank)
        if mb_only:
            ctx.select_allreduce(args.allreduce if args.allreduce == "mailbox-step" else "mailbox")
            halo_x = "mailbox"
        else:
            ctx.select_allreduce(args.allreduce if args.allreduce in ("mailbox", "mailbox-step") and
                                 ctx.comm_info()["allreduce"] in MAILBOX_KINDS else "rccl")
    fused = variant in ("fused", "pipelined")
    pipelined = variant == "pipelined"
    # the K timed steps are captured as one hipGraph before the clock starts (kernels, halo
    # send/recv, allreduces, per-kernel events as graph nodes) and replayed once inside it
    # One GPU, fused step: the timed region has exactly one kernel launch per step, so the two
    # HIP events bracketing the region (always recorded on the library stream) time the kernel:
    # region / K = average launch duration including the inter-launch gap (a conservative kernel
    # time).  Per-launch events there would add an event packet between consecutive kernels
    # (measured: 4590 vs 4830 steps/s).  Two-kernel steps keep per-kernel events.
    region = world == 1 and variant == "fused" and args.kernel_events != "per-launch"
    kev = not args.no_kernel_events and not region
    eager = args.launch == "eager" or (args.launch == "auto" and world == 1)
    # graph replay (the N > 1 default): the timed graph carries no per-launch events; a second,
    # short graph with per-launch event nodes is replayed after the timed region for the kernel
    # timing, so the event packets do not sit between the timed kernels
    K2 = min(K, 20) if kev and not eager else 0
    ws = eigmi.LanczosWorkspace(M, W + K + K2, seed=123, fused=variant == "fused", pipelined=pipelined)
    if W:
        ws.step(W)
    graph = False if eager else ws.capture(K, timed=kev and K2 == 0)
    k0, L0 = ws.info()
    barrier()
    ctx.sync()
    t0 = time.perf_counter()
    tim = ws.step(K, timed=kev) if eager else ws.replay()
    ctx.sync()
    barrier()
    dt = max_over_ranks(time.perf_counter() - t0)
    k1, L1 = ws.info()
    # fused: a launch whose norm prediction is unsound repairs instead of stepping (k_spmv.hip
    # fused_begin) and the workspace tops the launches up until K steps are done
    repairs = (L1 - L0) - (k1 - k0)
    region = region and repairs == 0
    if K2:
        # kernel timing pass (outside the timed region): K2 more steps, per-launch event nodes
        ws.capture(K2, timed=True)
        tim_k = ws.replay()
        ctx.sync()
    else:
        tim_k = tim
    alpha, beta = ws.tridiag()
    ok = bool(np.all(np.isfinite(alpha)) and np.all(beta[1:] > 0))

    # dominant kernel: the step kernel (fused) or the SpMV kernel (classic), HIP events on the
    # library stream around every launch of the timed region
    # algorithmic bytes per launch are those of the matrix image the kernel streams (DESIGN.md
    # section 5): the symmetric band image moves 8 B per upper-band slot + a 1-B row mask, i.e.
    # fewer bytes than the survey's CSR count (12 B per nonzero), which is reported beside it
    kname, k1_bytes = M.lanczos_kernel_info(fused)
    csr_bytes = eigmi.bytes_lanczos_fused(cnt, nnz_local) if fused else eigmi.bytes_lanczos_k1(cnt, nnz_local)
    if pipelined:
        # timed launch = the SpMV of t_{k-1} (eig_mv's kernel) + the row kernel (32 B read + 24 B
        # written per row)
        kname = M.kernel("spmv") + "+k_lanczos_pipe"
        k1_bytes = eigmi.image_bytes(M, "spmv") + 56 * cnt
        csr_bytes = eigmi.bytes_spmv(cnt, nnz_local) + 56 * cnt
    k1_ms = (tim_k.spmv_ms / tim_k.spmv_launches if tim_k.spmv_launches else
             (tim.total_ms / K if region and K else None))
    roofline = None
    if k1_ms:
        ach = k1_bytes / (k1_ms * 1e-3) / 1e9
        tr = committed_traffic(kernel_instance(M, kname), N, world, build, args.image)
        roofline = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": tr[0] if tr else None,
                    "traffic_source": tr[1] if tr else None,
                    "traffic_same_build": tr[2] if tr else None,
                    "traffic_GBs": round(tr[0] / (k1_ms * 1e-3) / 1e9, 1) if tr else None,
                    "traffic_frac": round(tr[0] / (k1_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if tr else None,
                    "kernel": kernel_instance(M, kname), "bytes_per_launch": k1_bytes,
                    "avg_launch_us": round(k1_ms * 1e3, 2),
                    "launch_timing": ("region events / K (one launch per step; includes the inter-launch gap)"
                                      if region else
                                      f"HIP event nodes around every launch of a {K2}-step replay after the timed one"
                                      if K2 else "HIP events around every launch"),
                    # the same launch priced at the survey's CSR byte count
                    "csr_bytes_per_launch": csr_bytes,
                    "csr_equiv_GBs": round(csr_bytes / (k1_ms * 1e-3) / 1e9, 1)}
    step_bytes = eigmi.bytes_lanczos_step(n, nnz_total)
    value = K / dt
    # outside the timed region: the standalone SpMV (eig_mv = BCRSMatrix::mv) on the same image, and
    # the measured HBM copy rate the roofline is also quoted against
    spmv = None
    copy_GBs = None
    if rank == 0 and world == 1:
        x = M.window_vector(np.random.default_rng(0).standard_normal(cnt))
        y = M.window_vector()
        M.mv_timed(x, y, 3)
        mv_ms = min(M.mv_timed(x, y, 20) for _ in range(3))
        ib = eigmi.image_bytes(M, "spmv")
        cb = eigmi.bytes_spmv(n, nnz_total)
        spmv = {"kernel": M.kernel("spmv"), "us": round(mv_ms * 1e3, 2), "bytes": ib,
                "GBs": round(ib / (mv_ms * 1e-3) / 1e9, 1), "frac": round(ib / (mv_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "csr_bytes": cb, "csr_equiv_GBs": round(cb / (mv_ms * 1e-3) / 1e9, 1)}
        x.free()
        y.free()
    sides = {}
    if rank == 0 and world == 1 and args.side_steps > 0:
        # the same step on the other images of the same matrix (side numbers: never value / roofline)
        def side_traffic(ki):
            return committed_traffic(ki, N, world, build, args.image)
        for img, key in (("csr", "csr"), ("uniform", "stencil_shortcut")):
            if img != args.image:
                sides[key] = side_image(ctx, rp, c, v, img, args.side_steps, n, nnz_total, traffic=side_traffic)
        if args.general_steps > 0 and args.matrix == "poisson":
            sides["general"] = side_general(ctx, N, args.general_steps, side_traffic)
    if rank == 0:
        copy_GBs = eigmi.stream_copy_GBs(ctx)
        if spmv:
            spmv["frac_vs_measured_copy"] = round(spmv["GBs"] / copy_GBs, 4)
        if roofline:
            roofline["measured_copy_GBs"] = round(copy_GBs, 1)
            roofline["frac_vs_measured_copy"] = round(roofline["achieved"] / copy_GBs, 4)
    out = {
        "metric": "Lanczos iters/sec + achieved SpMV HBM GB/s, 3D Poisson 256^3",
        "value": round(value, 3),
        "unit": "iters/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": round(dt / K * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("synthetic (generated 7-point Poisson matrix" if args.matrix == "poisson" else
                 "synthetic (generated variable-coefficient 7-point matrix, eig_gen kind 8") +
                ", mt19937 seed-123 start vector)",
        "config": {"workload": f"3D {'Poisson' if args.matrix == 'poisson' else 'variable-coefficient'} 7-pt "
                               f"{N}^3 Lanczos 3-term step, no re-orthogonalisation ({VARIANT_NAME[variant]})",
                   "N": N, "n": n, "nnz": nnz_total, "matrix": args.matrix, "image": args.image,
                   "matrix_image": image_name(M),
                   "parallelism": (f"row-partition z-slabs x{world} "
                                   f"({'halo mailbox' if halo_x == 'mailbox' else 'RCCL halo'}, {halo_mode} launch, "
                                   f"{ctx.comm_info()['allreduce']} allreduce)") if world > 1 else
                                  ("single GPU, one-rank RCCL allreduce per step" if args.comm_self else "single GPU")},
        # SURVEY 8(d)'s CSR step bytes (12 nnz + 4(n+1) + 48 n) / step time: an equivalent rate, not
        # HBM traffic (the band image streams fewer bytes; roofline.* prices the kernel's own bytes)
        "step_csr_equiv_GBs": round(step_bytes / (dt / K) / 1e9, 1),
        "roofline": roofline,
        "spmv_hbm_gbs": roofline["achieved"] if roofline else None,
        # eig_mv alone (y = A x on the same image, 20 launches x 3, best average), beside the step
        "spmv": spmv,
        # N = 1: the same fused step on the SELL / CSR image (SURVEY 8(d)'s CSR bytes are what it streams at
        # most) and on the constant-coefficient shortcut (no matrix bytes) -- side numbers only
        **sides,
        # device time of the K steps: fused SpMV launches vs the rest (update kernel, allreduces)
        "device_ms": {"total": round(tim.total_ms, 3),
                      "spmv": round(tim.total_ms if region else tim.spmv_ms, 3),
                      "rest": round(0.0 if region else tim.total_ms - tim.spmv_ms, 3)},
        "recurrence_finite": ok,
        "fused_repairs": repairs if fused else None,
        "variant": variant,
        # auto at N > 1: ms per step of each one-reduction variant in the trial (max over ranks)
        "variant_trial_ms": ({k: (v if v != float("inf") else None) for k, v in trial.items()} if trial else None),
        "launch": "hipGraph replay of the K steps" if graph else "eager",
        # the communicator the timed steps ran on (RCCL saw nranks ranks) and its transport check
        "comm": comm_summary(ctx, world, ab_check),
        "build": build,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cv, cdt, rel = cpu_baseline(N, rp, c, v, args.cpu_steps, alpha, fused)
        out["cpu_baseline"] = {"value": round(cv, 4), "unit": "iters/s", "cores": 1, "kind": "port",
                               "sample": f"{args.cpu_steps} Lanczos steps on the same {N}^3 matrix and start "
                                         f"vector, oracle/oracle.cc built -O3 -march=x86-64-v3 "
                                         f"(liboracle_fast.so), single thread ({cdt:.1f} s)",
                               "alpha_max_rel_diff_vs_gpu": rel, "cpu_model": cpu_model()}
        sv, sdt, srel = scipy_crosscheck(N, rp, c, v, args.scipy_steps, alpha)
        out["cpu_baseline"]["scipy_crosscheck"] = {
            "value": round(sv, 4), "unit": "iters/s", "cores": 1,
            "sample": f"{args.scipy_steps} plain Lanczos steps with scipy.sparse CSR matvec + numpy BLAS-1 "
                      f"(ARPACK's operator in scipy eigsh), same matrix and start vector ({sdt:.1f} s)",
            "alpha_max_rel_diff_vs_gpu": srel}
        P = args.cpu_replicas
        usable = len(os.sched_getaffinity(0))
        if P is None:
            # the GPU box grants 16 CPUs per GPU (gpurun's process guard; nproc reports the whole
            # machine), and each replica holds its own 1.9 GB matrix + vectors
            P = min(16, usable)
        if P > 0:
            pv, pdt = cpu_replicas(N, rp, c, v, args.cpu_replica_steps, fused, P)
            out["cpu_baseline"]["replicas"] = {
                "value": round(pv, 4) if pv else None, "unit": "iters/s", "cores": P,
                "sample": f"{P} concurrent replicas x {args.cpu_replica_steps} steps, each on its own "
                          f"{N}^3 matrix (the reference's numthreads mode, .cc:754-760) ({pdt:.1f} s)",
                "cap": f"{P} of {usable} visible cores (nproc {os.cpu_count()}): the box allots 16 CPUs per GPU"}
    if rank == 0:
        os.write(out_fd, (json.dumps(out) + "\n").encode())
    ws.close()
    M.close()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
