"""The one stream / queue / step-mode policy of a training process.

Every entry point (bench.py, the per-family trainers, the Hourglass click CLI, and each rank that
``torch.distributed.run`` starts for them) calls :func:`configure` BEFORE HIP initialises -- this
module imports neither torch nor any other part of the package, so it can run before ``import
torch``. ``configure`` decides, once per process:

* the step mode: HIP-graph replay of the whole step ("graph") or eager, from :data:`PREFERRED`
  (measured same-box 1-GPU rates, README "Results") unless the caller forces one;
* ``GPU_MAX_HW_QUEUES``: eager steps get 8 hardware queues (compute, weight-gradient side stream and
  RCCL's streams each on a queue of their own -- with HIP's default 4 the side stream shared the
  compute queue under RCCL and serialised: world-1 RCCL ResNet-50 12,960 img/s without it, 13,690
  with it and 8 queues); captured steps keep HIP's default 4 (a graph whose side-stream branches
  land on queues of their own replayed 24-35 % slower, profiles/wgrad_side_stream_ab.txt). A larger
  value already in the environment is kept; ``DV_KEEP_HW_QUEUES=1`` keeps any value (A/B runs).

:func:`side_policy` then resolves where weight gradients run (ops/conv.py reads it, not the
environment): on the side stream in single-process eager steps; under a process group only with
>= 8 queues; inside a capture only with < 8 queues. The env switches below override single fields
for same-box A/B runs and are read here only:

=========================  =====================================================================
DV_WGRAD_SIDE              0 off, 3x3 only R*S > 1 convs, else every conv (default)
DV_WGRAD_SIDE_COMM         side (bucket all-reduces issue from the side stream) | flush
DV_WGRAD_SIDE_OPTOUT       0 ignores the models' no_wgrad_side() opt-outs (Hourglass, MobileNet)
DV_WGRAD_SIDE_DP           0 / 1 forces the under-a-process-group decision
DV_WGRAD_SIDE_GRAPH        0 / 1 forces the inside-a-capture decision
DV_KEEP_HW_QUEUES          1 leaves GPU_MAX_HW_QUEUES as the caller set it
=========================  =====================================================================

(Per-kernel A/B switches that do not change the process's stream / queue layout stay with their
kernels in ops/conv.py: DV_SUBPIXEL_CONC -- a strided dgrad's parity parts on streams of their own,
off in deterministic mode; DV_DGRAD_SPLIT; DV_FIN_BNR.)

Reference: the reference launches every trainer one way (R/ResNet/pytorch/train.py:353-355
DataParallel over all GPUs; R/YOLO/tensorflow/train.py:281-294 MirroredStrategy).
"""
from __future__ import annotations

import os

# model -> step mode measured faster on one MI355X (README "Results"; bench.py eager vs --graph):
#   resnet50 eager 13,865 vs graph 13,326 img/s; mobilenet1 graph 25,891 vs eager host-bound;
#   shufflenet1 graph 14,336 vs eager 7,271; yolov3 graph 1,165 vs eager 950-1,250 (box-dependent);
#   hourglass graph 1,428 vs eager 823-894. The big-map classifiers (VGG, AlexNet, Inception, the
#   ResNets) are device-bound and keep eager; the small / many-kernel models are host-bound.
PREFERRED = {
    "resnet18": "eager", "resnet34": "eager", "resnet50": "eager", "resnet101": "eager", "resnet152": "eager",
    "vgg16": "eager", "vgg19": "eager", "alexnet1": "eager", "alexnet2": "eager", "alexnet": "eager",
    "inception1": "eager", "inception3": "eager",
    "mobilenet1": "graph", "mobilenet2": "graph", "shufflenet1": "graph",
    "yolov3": "graph", "hourglass": "graph", "centernet": "graph",
    "lenet5": "eager", "lenet": "eager", "dcgan": "eager", "cyclegan": "eager",
}
EAGER_QUEUES = 8
HIP_DEFAULT_QUEUES = 4


def preferred_graph(model: str | None) -> bool:
    """True when ``model``'s captured step measured faster than its eager step (unknown: eager)."""
    return PREFERRED.get((model or "").lower(), "eager") == "graph"


def hw_queues(env=None) -> int:
    env = os.environ if env is None else env
    try:
        return int(env.get("GPU_MAX_HW_QUEUES", str(HIP_DEFAULT_QUEUES)))
    except ValueError:
        return HIP_DEFAULT_QUEUES


def queues_env(env, graph: bool) -> None:
    """Set ``env``'s GPU_MAX_HW_QUEUES for a step mode (see the module docstring)."""
    if not graph and env.get("DV_KEEP_HW_QUEUES") != "1" and hw_queues(env) < EAGER_QUEUES:
        env["GPU_MAX_HW_QUEUES"] = str(EAGER_QUEUES)


def configure(model: str | None = None, graph: bool | None = None, env=None) -> bool:
    """Resolve the step mode (``graph`` None -> :data:`PREFERRED`) and set this process's (or a child
    environment's) hardware-queue count for it; returns the graph decision. Call before HIP
    initialises: the runtime reads GPU_MAX_HW_QUEUES once, at its first call."""
    env = os.environ if env is None else env
    g = preferred_graph(model) if graph is None else bool(graph)
    queues_env(env, g)
    env["DV_STEP_MODE"] = "graph" if g else "eager"
    return g


_FLAG = {"0": False, "1": True}


def side_policy(env=None) -> dict:
    """Where weight gradients run, resolved from the queue count and the A/B switches."""
    env = os.environ if env is None else env
    q = hw_queues(env)
    return {
        "hw_queues": q,
        "wgrad_side": {"0": False, "3x3": "3x3"}.get(env.get("DV_WGRAD_SIDE", "1"), "all"),
        "comm": env.get("DV_WGRAD_SIDE_COMM", "side"),
        "optout": env.get("DV_WGRAD_SIDE_OPTOUT", "1") != "0",
        "under_dp": _FLAG.get(env.get("DV_WGRAD_SIDE_DP", ""), q >= EAGER_QUEUES),
        "in_capture": _FLAG.get(env.get("DV_WGRAD_SIDE_GRAPH", ""), q < EAGER_QUEUES),
    }


def describe(env=None, world_size: int | None = None) -> dict:
    """The resolved policy of this process as one flat record (printed by ``bench.py --policy``)."""
    env = os.environ if env is None else env
    sp = side_policy(env)
    ws = int(env.get("WORLD_SIZE", "1")) if world_size is None else world_size
    mode = env.get("DV_STEP_MODE", "eager")
    side = bool(sp["wgrad_side"])
    # ops/conv.py: ctx.wside = side and not (process group and not under_dp) and not (capturing and
    # not in_capture)
    active = side and (ws <= 1 or sp["under_dp"]) and (mode != "graph" or sp["in_capture"])
    return {"mode": mode, "world_size": ws, "hw_queues": sp["hw_queues"], "wgrad_side": sp["wgrad_side"],
            "wgrad_side_active": active, "side_comm": sp["comm"] if active and ws > 1 else None,
            "optout": sp["optout"]}
