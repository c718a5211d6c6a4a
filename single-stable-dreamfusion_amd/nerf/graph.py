"""HIP-graph capture of the SDS train step.

The reference's train step (nerf/utils.py:693-715 -> train_step :337-404 ->
NeRFRenderer.run_cuda, renderer.py:446-559) is ~300 small launches plus one
host synchronisation (the march's `step_counter[0].item()`,
raymarching.py:224).  On MI355X the kernels of one 128x128 step take ~2.7 ms
while the eager step takes ~4.7 ms: the rest is launch latency and the drain
after the sync.  Here the step is captured once per (shading, resolution) and
replayed:

* the march runs in its device-count form (raymarching.march_rays_train_dev):
  capacity-sized sample buffers, the live count stays on the GPU, every
  per-sample consumer (fused grid field, mixed compositing, their backwards)
  stops at it;
* the native step's graph (nerf/native_step.py) holds render -> SDS
  gradient -> regulariser -> the whole backward, the embedding-gradient
  scatter included, and GradScaler + Adam as well (device learning rates
  written by the prologue launch); with data parallelism over RCCL the flat
  in-place all-reduce of the gradient bucket and the 1/world scaling sit
  in the graph before Adam, so each rank replays ONE graph per step (a gloo
  group, not capturable, ends the graph at the gradients and the exchange
  and Adam follow eagerly);
* the autograd form's graph ends at the feature gradients; the embedding
  scatter is launched eagerly after each replay, then the optimizer step;
* kernel timing (bench.py) never reaches into a graph: it runs the native
  body eagerly under a kernel timer (step_timed()), the same launches the
  graph replays.

The albedo shading is captured in both forms; the textureless / lambertian
steps (finite-difference normals, csrc/shade.hip) only as the native step.  RNG draws inside the graph (march noise, background colour, light
direction, timestep, SDS noise) use torch's graph-safe Philox offsets, so
every replay draws fresh numbers.
"""
import torch

import _dfhip
from . import field as _field
from . import native_step as _native


class GraphedTrainStep:
    def __init__(self, trainer, data, shading, ambient_ratio, text_z, stream, allow_native=True):
        self.trainer = trainer
        self.shading, self.ambient_ratio = shading, ambient_ratio
        self.H, self.W = data["H"], data["W"]
        # the albedo step as native launches without autograd (nerf/native_step.py)
        self.native = None
        if (trainer.native_step and allow_native and "pose" in data and "intrinsics" in data
                and _native.eligible(trainer, shading)):
            self.native = _native.NativeAlbedoStep(trainer, self.H, self.W, shading,
                                                   ambient_ratio)
            self.rays_o = self.native.rays_o.view(1, -1, 3)
            self.rays_d = self.native.rays_d.view(1, -1, 3)
        else:
            self.rays_o = data["rays_o"].detach().clone()
            self.rays_d = data["rays_d"].detach().clone()
        self.text_z = text_z.detach().clone()
        self._text_src = text_z.data_ptr()  # prompt tensor currently in self.text_z
        self.stream = stream
        self.graph = torch.cuda.CUDAGraph()
        self.optimizer_in_graph = False
        self.deferred = []
        self.grads = None
        self.counter = None
        self.loss = None

    def _body(self, static):
        t = self.trainer
        with torch.autocast("cuda", enabled=t.amp, dtype=t.amp_dtype):
            _, _, loss = t.train_step(static, shading=self.shading,
                                      ambient_ratio=self.ambient_ratio, text_z=self.text_z)
        t.backward_only(loss)
        return loss

    def _capture_native(self, data):
        nat = self.native
        t = self.trainer
        model = t.model
        timer = _dfhip.set_kernel_timer(None)  # no event records inside the graph
        try:
            # the optimizer step joins the graph: on one GPU directly, with data
            # parallelism behind the flat RCCL all-reduce of the gradient
            # bucket (captured too: one replay per step on every rank)
            self.optimizer_in_graph = False
            collective = t.graph_collective()
            if t.world_size == 1 or collective:
                adam = t.native_adam()
                if adam:
                    nat.attach_optimizer(adam)
                    if collective:
                        nat.attach_allreduce(t.world_size)
                    self.optimizer_in_graph = True
            self.load(data, self.text_z)
            self.stream.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self.stream):
                # dry run (first-use setup outside the capture); neither the
                # optimizer nor the all-reduce runs.  The communicator is
                # already up (Trainer's rank-0 parameter broadcast), and a
                # step that captures must issue exactly as many collectives as
                # a step that replays (one, inside the graph): ranks that
                # capture a (shading, H, W) key on different steps then still
                # pair their collectives step for step.
                nat.body()
                nat.embedding_backward()
            with torch.cuda.graph(self.graph, stream=self.stream):
                self.loss = nat.body()
                nat.embedding_backward()
                if self.optimizer_in_graph:
                    if nat.dp_world is not None:
                        nat.allreduce_tail()
                    nat.optimizer_tail()
            torch.cuda.current_stream().wait_stream(self.stream)
        finally:
            _dfhip.set_kernel_timer(timer)
        model.local_step += 1  # as run_cuda's step in the autograd capture
        model.last_counter = nat.counter
        self.counter = nat.counter
        self.deferred = []
        self.grads = list(nat.grads)

    def capture(self, data=None):
        """Record the step (nothing of it executes until replay()).

        First one untimed dry run of the same code on the capture stream (its
        gradients are dropped, no optimizer step): the BLAS / MIOpen libraries
        set up per-stream state on first use, which must not happen inside the
        capture (HIP then faults when the capture ends)."""
        if self.native is not None:
            return self._capture_native(data)
        t = self.trainer
        model = t.model
        params = [p for p in model.parameters() if p.requires_grad]
        static = {"H": self.H, "W": self.W, "rays_o": self.rays_o, "rays_d": self.rays_d,
                  "dir": None}
        model.device_count_march = True
        timer = _dfhip.set_kernel_timer(None)  # no event records inside the graph
        step0 = model.local_step
        # the graph's march counts into a private row; every replay's count is
        # copied into the row of its own step (Trainer)
        step_counter = model.step_counter
        model.step_counter = torch.zeros_like(step_counter)
        try:
            self.stream.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self.stream):
                t.optimizer.zero_grad(set_to_none=True)
                with _field.defer_embedding_backward():
                    self._body(static)
                t.optimizer.zero_grad(set_to_none=True)
            model.local_step = step0
            with _field.defer_embedding_backward() as deferred:
                with torch.cuda.graph(self.graph, stream=self.stream):
                    self.loss = self._body(static).detach()
            torch.cuda.current_stream().wait_stream(self.stream)
        finally:
            model.device_count_march = False
            model.step_counter = step_counter
            _dfhip.set_kernel_timer(timer)
        self.deferred = list(deferred)
        self.counter = model.last_counter
        # gradients written by the graph (the embedding's comes from the
        # deferred launch), re-attached after every replay
        emb = getattr(model, "encoder", None)
        self.grads = []
        for p in params:
            g = p.grad
            if g is None and emb is not None and p is emb.embeddings and self.deferred:
                g = self.deferred[0][1]
            self.grads.append((p, g))

    def load(self, data, text_z):
        """This step's camera rays (made straight into the graph's input buffers
        from a host pose when the batch has one) and prompt embedding."""
        if self.native is not None:
            t = self.trainer
            self.native.prologue(data["pose"], data["intrinsics"],
                                 int(t.opt.seed) * 1000003 + int(t.local_rank), t.global_step)
            return
        if "pose" in data and "rays_o" not in data:
            from .utils import get_rays_host_pose
            get_rays_host_pose(data["pose"], data["intrinsics"], self.H, self.W, None,
                               out=(self.rays_o, self.rays_d))
        else:
            self.rays_o.copy_(data["rays_o"], non_blocking=True)
            self.rays_d.copy_(data["rays_d"], non_blocking=True)
        if text_z.data_ptr() != self._text_src:
            self.text_z.copy_(text_z, non_blocking=True)
            self._text_src = text_z.data_ptr()

    def replay(self):
        """Run the captured part, then (autograd form) the deferred embedding
        backward; leaves every trainable parameter's .grad set (and, with
        optimizer_in_graph, the parameters already updated)."""
        self.graph.replay()
        for launch, _ in self.deferred:
            launch()
        for p, g in self.grads:
            p.grad = g

    def step_timed(self):
        """The native step's launches run eagerly (no graph) under whatever
        kernel timer is installed: the same kernels, arguments and buffers the
        replay runs, each in its timed region (bench.py kernel-timing pass).
        Call after load(); the optimizer runs when the graph holds it."""
        nat = self.native
        if nat is None:
            raise RuntimeError("step_timed: only the native step has an eager twin")
        nat.body()
        nat.embedding_backward()
        if self.optimizer_in_graph:
            if nat.dp_world is not None:
                nat.allreduce_tail()
            nat.optimizer_tail()
        for p, g in self.grads:
            p.grad = g


class BucketedModuleStep:
    """The train step through the reference-API modules (GridEncoder, the MLP
    module, trunc_exp / sigmoid, composite_rays_train, the ray head: the
    Trainer's autograd body with `model.fused_field = False`) in the
    reference's own structure — the march counts its samples and the host
    reads the count (`step_counter[0].item()`, raymarching.py:224) — with the
    rest of the step replayed from a HIP graph instead of launched op by op.

    Per step: the camera rays, near / far, march noise and the staged march
    (count + emit into persistent buffers) run eagerly; the host reads the
    sample count M, as the reference does, and picks the smallest row bucket
    Mb >= M (geometric, ratio 1.25, multiples of 4096); rows [M, Mb) of the
    samples are zeroed, and the graph captured for Mb replays field ->
    compositing -> head -> loss -> backward on the [0, Mb) views.  Every
    per-sample op therefore runs on Mb rows (<= 1.25 M) instead of the
    capacity N * max_steps, and the modules that honour the device live-row
    count (GridEncoder, the MLP kernels, the compositing) stop at M.  The
    gradients are copied into one flat bucket at the end of the graph, so the
    optimizer sees the same gradient buffers whatever the bucket.  A graph is
    captured per bucket on first use (a few over a run)."""

    RATIO = 1.25
    MIN_ROWS = 1 << 16
    ALIGN = 4096

    def __init__(self, trainer, H, W, shading, ambient_ratio, stream):
        import _raymarching
        from .utils import flat_grad_bucket_
        t = trainer
        m = t.model
        dev = t.device
        self.trainer, self.shading, self.ambient_ratio = t, shading, ambient_ratio
        self.H, self.W = int(H), int(W)
        N = self.N = self.H * self.W
        self.max_steps = int(t.opt.max_steps)
        cap = self.cap = N * self.max_steps
        f32 = dict(device=dev, dtype=torch.float32)
        self.rays_o = torch.empty(1, N, 3, **f32)
        self.rays_d = torch.empty(1, N, 3, **f32)
        self.nears = torch.empty(N, **f32)
        self.fars = torch.empty(N, **f32)
        self.noises = torch.empty(N, **f32)
        self.rays = torch.empty(N, 3, device=dev, dtype=torch.int32)
        self.counter = torch.zeros(2, device=dev, dtype=torch.int32)
        self.block_sums = torch.empty(_raymarching.march_rays_train_scratch_ints(N), device=dev,
                                      dtype=torch.int32)
        self.stage = torch.empty(_raymarching.march_rays_train_stage_floats(N, self.max_steps),
                                 **f32)
        self.xyzs = torch.empty(cap, 3, **f32)
        self.dirs = torch.empty(cap, 3, **f32)
        self.deltas = torch.empty(cap, 2, **f32)
        self.params = [p for p in m.parameters() if p.requires_grad]
        self.grad_bucket = flat_grad_bucket_(self.params)
        self.grad_views = [p.grad for p in self.params]
        self.stream = stream
        self.pool = torch.cuda.graph_pool_handle()
        self.graphs = {}  # bucket rows -> (graph, loss)
        self.text_z = None
        self._text_src = None
        self.last_rows = None
        # (GraphedTrainStep's attributes bench.py reads)
        self.native = None
        self.optimizer_in_graph = False

    def bucket(self, m):
        b = self.MIN_ROWS
        while b < m:
            b = -(-int(b * self.RATIO) // self.ALIGN) * self.ALIGN
        return min(b, self.cap)

    def march(self, data):
        """The eager part: rays, near / far, noise, the staged march; returns
        the sample count read on the host (the reference's sync)."""
        import raymarching
        import _raymarching
        from .utils import get_rays_host_pose
        m = self.trainer.model
        if "pose" in data and "rays_o" not in data:
            get_rays_host_pose(data["pose"], data["intrinsics"], self.H, self.W, None,
                               out=(self.rays_o, self.rays_d))
        else:
            self.rays_o.copy_(data["rays_o"], non_blocking=True)
            self.rays_d.copy_(data["rays_d"], non_blocking=True)
        ro, rd = self.rays_o.view(-1, 3), self.rays_d.view(-1, 3)
        # the train path passes no min_near -> the op's default 0.2 (renderer.py:458)
        _raymarching.near_far_from_aabb(ro, rd, m.aabb_train, self.N, 0.2, self.nears,
                                        self.fars)
        torch.rand(self.N, out=self.noises)  # perturb=True in train_step
        self.counter.zero_()
        dt_gamma = float(self.trainer.opt.dt_gamma)
        _raymarching.march_rays_train_count_staged(
            ro, rd, m.density_bitfield, m.bound, dt_gamma, self.max_steps, self.N, m.cascade,
            m.grid_size, self.nears, self.fars, self.rays, self.counter, self.noises,
            self.block_sums, self.stage)
        _raymarching.march_rays_train_emit_staged(
            rd, self.max_steps, self.N, self.cap, self.xyzs, self.dirs, self.deltas, self.rays,
            self.block_sums, 0, self.stage)
        del raymarching
        return int(self.counter[0].item())  # D2H sync (raymarching.py:224)

    def _premarched(self, rows):
        """The march outputs as run_cuda consumes them: [0, rows) views that
        carry the device live-row count; rays ray-ordered."""
        from raymarching.raymarching import LIVE_ROWS_ATTR, _ORDERED_ATTR
        xyzs, dirs, deltas = self.xyzs[:rows], self.dirs[:rows], self.deltas[:rows]
        for v in (xyzs, dirs, deltas, self.rays):
            setattr(v, LIVE_ROWS_ATTR, self.counter[:1])
        setattr(self.rays, _ORDERED_ATTR, True)
        return (self.nears, self.fars, xyzs, dirs, deltas, self.rays)

    def _body(self, rows):
        t = self.trainer
        model = t.model
        static = {"H": self.H, "W": self.W, "rays_o": self.rays_o, "rays_d": self.rays_d,
                  "dir": None}
        model.premarched = self._premarched(rows)
        try:
            with torch.autocast("cuda", enabled=t.amp, dtype=t.amp_dtype):
                _, _, loss = t.train_step(static, shading=self.shading,
                                          ambient_ratio=self.ambient_ratio, text_z=self.text_z)
            t.backward_only(loss)
        finally:
            model.premarched = None
        # the gradients into the flat bucket the optimizer steps: one
        # multi-tensor copy launch (per-tensor copies were 12 blit launches,
        # ~58 us per step)
        dst, src = [], []
        for p, v in zip(self.params, self.grad_views):
            if p.grad is not None and p.grad is not v:
                dst.append(v)
                src.append(p.grad)
        if dst:
            torch._foreach_copy_(dst, src)
        return loss

    def _capture(self, rows):
        t = self.trainer
        timer = _dfhip.set_kernel_timer(None)  # no event records inside the graph
        try:
            self.stream.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self.stream):
                # dry run: library first-use setup outside the capture
                for p in self.params:
                    p.grad = None
                self._body(rows)
            for p in self.params:
                p.grad = None
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=self.stream, pool=self.pool):
                loss = self._body(rows).detach()
            torch.cuda.current_stream().wait_stream(self.stream)
        finally:
            _dfhip.set_kernel_timer(timer)
            for p, v in zip(self.params, self.grad_views):
                p.grad = v
        self.graphs[rows] = (g, loss)
        return self.graphs[rows]

    def step(self, data, text_z):
        """One step: the eager march, the count, the bucket's graph.  Leaves
        every parameter's .grad a view of the flat bucket.  Returns the loss."""
        if self.text_z is None:
            self.text_z = text_z.detach().clone()
            self._text_src = text_z.data_ptr()
        elif text_z.data_ptr() != self._text_src:
            self.text_z.copy_(text_z, non_blocking=True)
            self._text_src = text_z.data_ptr()
        M = self.march(data)
        rows = self.bucket(max(M, 1))
        self.last_rows = (M, rows)
        # rows past the count: zeros (finite inputs for the per-row torch ops)
        if rows > M:
            self.xyzs[M:rows].zero_()
            self.dirs[M:rows].zero_()
            self.deltas[M:rows].zero_()
        g = self.graphs.get(rows)
        if g is None:
            g = self._capture(rows)
        g[0].replay()
        for p, v in zip(self.params, self.grad_views):
            p.grad = v
        return g[1]

    def precapture(self, max_rows):
        """Capture the graphs of every bucket up to bucket(max_rows) now (the
        bench does this after its warm-up, so no capture lands in a timed
        region).  The dry runs use the last step's march; their gradients are
        overwritten by the next replay."""
        b = self.MIN_ROWS
        top = self.bucket(max_rows)
        while True:
            if b not in self.graphs:
                self._capture(b)
            if b >= top:
                break
            b = self.bucket(b + 1)
