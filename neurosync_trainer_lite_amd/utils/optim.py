"""Fused Adam (coupled L2) + global-norm clip over the engine's flat parameter arena.

Drop-in for ``torch.optim.Adam(model.parameters(), lr, weight_decay)`` as built at
/root/reference/utils/model_utils.py:11, including the state_dict format
({'state': {i: {'step', 'exp_avg', 'exp_avg_sq'}}, 'param_groups': [...]}) so
reference checkpoints load and ours load into torch.optim.Adam.  One
``nstl_sumsq`` + one ``nstl_adam_step`` launch replace clip_grad_norm_'s
per-tensor norms and Adam's ~5 foreach passes (training_utils.py:73-74), and the
norm stays on the device (the reference syncs 344 ``.item()``s per step).
"""
import os

import torch

from .. import _hip as K

N_PARTIAL = 1024


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False, *,
                 foreach=None, maximize=False, capturable=False, differentiable=False, fused=None,
                 decoupled_weight_decay=False):
        if amsgrad or maximize or decoupled_weight_decay:
            raise NotImplementedError("amsgrad/maximize/decoupled_weight_decay are not used by the reference")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad, maximize=maximize,
                        foreach=foreach, capturable=capturable, differentiable=differentiable, fused=fused,
                        decoupled_weight_decay=decoupled_weight_decay)
        super().__init__(params, defaults)
        if len(self.param_groups) != 1:
            raise NotImplementedError("FusedAdam supports one parameter group (as the reference uses)")
        self._engine = None
        self._nstl_step = 0
        self.last_norm = None
        self._comm = None            # parallel.ShardComm when sharded (ZeRO-1)
        self._moments_stale = False  # sharded: m/v outside this rank's shard are old
        # The caller's next use of the parameters is the model's forward (the
        # training loop sets this): the update is queued on a side stream in arena
        # ranges that the forward waits for stage by stage (Seq2SeqEngine.
        # queue_update), so it runs under the forward of earlier layers.  Results
        # are identical; any other reader of the parameters syncs first
        # (state_dict, module-level forwards, backward).
        # On by default since round 6 (NSTL_ADAM_OVERLAP=0: the update in order):
        # beside the 4-wave GEMMs (one wave per SIMD, 480 of 512 registers) the
        # update's 28-register waves co-reside, and the 228M step gains ~1 %
        # same-box (649.9k vs 643.6k frames/s, profiles/r6_adam_overlap_ab.txt).
        # Round 2 measured no gain beside the 8-wave ring GEMMs, which hold every
        # register of a SIMD (562.0k vs 561.3k).
        self.overlap_next_forward = False
        # The caller guarantees nothing writes the gradients between backward and
        # step() (train_one_epoch's own loop sets this): the clip norm may then
        # come from the weight-gradient GEMM epilogues' sums of squares.  Off by
        # default: drop-in code that averages or rescales p.grad in between (the
        # reference's multi-GPU path copies into p.grad.data,
        # utils/training_utils.py:235) gets the norm re-read from the arena.
        self.trust_backward_norm = False
        self._overlap_allowed = os.environ.get("NSTL_ADAM_OVERLAP", "1") == "1"
        self._upd_stream = None
        # why the data-parallel exchange left NSTL_DP=zero1_push for zero1, if it did
        # (attach_data_parallel at setup, ShardPusher.verify at the first step)
        self.dp_fallback = None
        # the first step's check of the pushed shard sums (ShardPusher.verify)
        self.dp_check = None

    # --------------------------------------------------------------- arena
    def _bind(self):
        params = self.param_groups[0]["params"]
        if self._engine is None:
            from ..engine import Seq2SeqEngine  # noqa: F401
            eng = _find_engine(params)
            if eng is None:
                raise RuntimeError("FusedAdam needs the parameters of a Seq2Seq whose engine is built "
                                   "(run one forward first, or build_model on a GPU)")
            names = {id(p): n for n, p in eng._params}
            if set(names) != {id(p) for p in params}:
                raise RuntimeError("FusedAdam must own exactly the Seq2Seq parameters")
            self._engine = eng
            self.m = torch.zeros_like(eng.p32)
            self.v = torch.zeros_like(eng.p32)
            self.partial = torch.empty(N_PARTIAL, dtype=torch.float32, device=eng.device)
            self.norm = torch.zeros(1, dtype=torch.float32, device=eng.device)
            self.coef = torch.ones(1, dtype=torch.float32, device=eng.device)
            for p in params:
                old = self.state.get(p, {})
                views = self._state_views(p)
                if "exp_avg" in old:  # state loaded before the arena existed
                    views["exp_avg"].copy_(old["exp_avg"].to(eng.device))
                    views["exp_avg_sq"].copy_(old["exp_avg_sq"].to(eng.device))
                self.state[p] = views
        return self._engine

    def _state_views(self, p):
        eng = self._engine
        o, k, shp = eng.offsets[eng.name_of[id(p)]]
        return {"step": torch.tensor(float(self._nstl_step)), "exp_avg": self.m[o:o + k].view(shp),
                "exp_avg_sq": self.v[o:o + k].view(shp)}

    # ---------------------------------------------------------------- step
    # ------------------------------------------------------------ sharding
    def shard(self, group=None):
        """Data-parallel ZeRO-1 (parallel.zero1_step): from now on step() reduce-
        scatters the gradients, clips with the global norm, updates this rank's
        1/n of the parameters and all-gathers the compute-dtype weights.  The f32
        master weights and Adam moments of the other shards go stale until
        consolidate() -- a collective every rank must call (e.g. before rank 0
        saves a checkpoint)."""
        from .. import parallel
        eng = self._bind()
        eng.ensure_bound()
        self._comm = parallel.ShardComm(eng.n_shardable, group)
        self._gs = torch.empty(self._comm.shard, dtype=torch.float32, device=eng.device)
        return self

    @torch.no_grad()
    def consolidate(self):
        """All-gather the f32 master weights and the Adam moments (collective)."""
        if self._comm is None:
            return
        eng = self._engine
        for t in (eng.p32, self.m, self.v):
            self._comm.all_gather(t[:eng.n_shardable])
        eng.master_stale = False
        self._moments_stale = False

    # ---------------------------------------------------------------- step
    @torch.no_grad()
    def step(self, closure=None, max_norm=None):
        """One Adam step; with ``max_norm`` the global-norm clip (clip_grad_norm_)
        is fused in front.  Returns the loss of ``closure`` (torch semantics)."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        eng = self._bind()
        eng.ensure_bound()
        g = self.param_groups[0]
        self._nstl_step += 1
        st = K.stream_of(eng.device)
        a = K.AdamArgs()
        a.lowp_dtype = K.dtype_code(eng.p16.dtype)
        a.lr, a.eps, a.weight_decay = g["lr"], g["eps"], g["weight_decay"]
        a.beta1, a.beta2 = g["betas"]
        a.step = self._nstl_step
        if max_norm is not None:
            a.sumsq_partial, a.n_partial, a.max_norm = self.partial.data_ptr(), N_PARTIAL, float(max_norm)
            a.norm_out = self.norm.data_ptr()

        def adam_fn(lo, n, grads, partial):
            a.p, a.g, a.m, a.v = (eng.p32[lo:].data_ptr(), grads.data_ptr(), self.m[lo:].data_ptr(),
                                  self.v[lo:].data_ptr())
            if eng.p16 is not eng.p32:
                a.p_lowp = eng.p16[lo:].data_ptr()
            a.n = n
            K.adam_step(a, stream=st)

        def sumsq_fn(grads, partial):
            if max_norm is not None:
                K.sumsq(grads, grads.numel(), partial, N_PARTIAL, stream=st)

        if self._comm is None and self.overlap_next_forward and self._overlap_allowed and closure is None:
            # clip coefficient on the current stream, the update in arena ranges on
            # the side stream (nstl_adam_step reads the coefficient: no LDS, so its
            # workgroups fit beside the forward's ring-GEMM workgroups)
            main = torch.cuda.current_stream(eng.device)
            sq = eng.take_sq_partials() if max_norm is not None and self.trust_backward_norm else None
            eng.invalidate_sq()
            if sq is not None:  # as below: the dW epilogues' partials + the rest of the arena
                parts, rp = self._norm_parts(sq), eng.sq_rest_partials
                o = sq.numel()
                for lo, hi in eng.norm_rest:
                    K.sumsq(eng.g32[lo:hi], hi - lo, parts[o:o + rp], rp, stream=st)
                    o += rp
                K.clip_coef(parts, o, max_norm, self.coef, self.norm, stream=st)
            elif max_norm is not None:
                sumsq_fn(eng.g32, self.partial)
                K.clip_coef(self.partial, N_PARTIAL, max_norm, self.coef, self.norm, stream=st)
            else:
                self.coef.fill_(1.0)
            if self._upd_stream is None:
                from ..parallel import side_stream
                self._upd_stream = side_stream(eng.device)
            side = self._upd_stream
            side.wait_stream(main)
            a.sumsq_partial, a.n_partial, a.norm_out, a.coef = None, 0, None, self.coef.data_ptr()

            def upd(lo, hi):
                a.p, a.g, a.m, a.v = (eng.p32[lo:].data_ptr(), eng.g32[lo:].data_ptr(), self.m[lo:].data_ptr(),
                                      self.v[lo:].data_ptr())
                if eng.p16 is not eng.p32:
                    a.p_lowp = eng.p16[lo:].data_ptr()
                a.n = hi - lo
                K.adam_step(a, stream=side.cuda_stream)
            eng.queue_update(upd, side)
            self._snapshot_norm(max_norm)
            return loss
        if self._comm is None:
            eng.sync_pending()
            red = eng.grad_reducer
            if red is not None and red.active and not red.consume():
                # replicated (NSTL_DP=allreduce) and no in-backward all-reduce
                # finished for these gradients (written by hand, or a backward that
                # raised): reduce them here
                import torch.distributed as dist
                eng.invalidate_sq()
                dist.all_reduce(eng.g32, op=dist.ReduceOp.SUM, group=red.group)
            sq = eng.take_sq_partials() if max_norm is not None and self.trust_backward_norm else None
            eng.invalidate_sq()
            if sq is not None:
                # the weight gradients' sums of squares came from the grouped dW
                # epilogues; nstl_sumsq covers the rest of the arena (head, embedding,
                # vectors), then one reduction gives the coefficient Adam reads
                parts, rp = self._norm_parts(sq), eng.sq_rest_partials
                o = sq.numel()
                for lo, hi in eng.norm_rest:
                    K.sumsq(eng.g32[lo:hi], hi - lo, parts[o:o + rp], rp, stream=st)
                    o += rp
                K.clip_coef(parts, o, max_norm, self.coef, self.norm, stream=st)
                a.sumsq_partial, a.n_partial, a.norm_out, a.coef = None, 0, None, self.coef.data_ptr()
                adam_fn(0, eng.numel, eng.g32, None)
            else:
                sumsq_fn(eng.g32, self.partial)
                adam_fn(0, eng.numel, eng.g32, self.partial)
            self._snapshot_norm(max_norm)
            return loss
        from .. import parallel
        if max_norm is None:
            self.partial.zero_()
        # the shard was summed in place during backward only if that backward's
        # reducer finished (not for gradients written by hand, or a backward that
        # raised): otherwise the step reduce-scatters as plain zero1 does
        red = eng.grad_reducer
        reduced = isinstance(red, parallel.GradShardReducer) and red.active and red.consume()
        sum_fn = gather_fn = None
        if isinstance(red, parallel.ShardPusher) and red.active:
            # the updated bf16 shard goes to the peers by the copy engines too
            # (unless this step's check of the pushed sums failed: then the
            # collective, as zero1)
            comm = self._comm

            def gather_fn(tensors):
                if red.failed:
                    for t in tensors:
                        comm.all_gather(t[:comm.numel])
                else:
                    red.all_gather(tensors)
        if isinstance(red, parallel.ShardPusher) and red.active and red.consume():
            # the other ranks' slices arrived in this rank's receive slots during
            # backward (copy engines): own + slots and the clip norm's partials
            # in one pass (nstl_shard_sum), instead of reduce-scatter + sumsq
            def sum_fn(g_shard, partial):
                K.shard_sum(eng.g32[comm.lo:comm.hi], red.slots(), red.n_slots, g_shard, partial, N_PARTIAL,
                            stream=st)
                if red.verify_pending:
                    red.verify(eng.g32, g_shard, partial, sumsq_fn)
                    self.dp_check = red.check
        parallel.zero1_step(self._comm, eng.g32, self._gs, self.partial, sumsq_fn, adam_fn,
                            [eng.p16] if eng.p16 is not eng.p32 else [eng.p32], tail=(eng.n_shardable, eng.numel),
                            reduced=reduced, sum_fn=sum_fn, gather_fn=gather_fn)
        if isinstance(red, parallel.ShardPusher) and red.failed:
            # every rank agreed the pushed sums were wrong (ShardPusher.verify):
            # from the next step on, the reduce-scatter
            red.close()
            eng.grad_reducer = None
            self.dp_fallback = "zero1_push -> zero1 (pushed shard sums differed from the reduce-scatter)"
        eng.master_stale = eng.p16 is not eng.p32
        self._moments_stale = True
        self._snapshot_norm(max_norm)
        return loss

    def _norm_parts(self, sq):
        """sq (the engine's dW partial buffer) followed by room for the rest-of-arena
        partials, as one contiguous buffer (sq is a prefix view of it)."""
        need = sq.numel() + self._engine.sq_rest_partials * len(self._engine.norm_rest)
        base = sq._base if sq._base is not None else sq
        if base.numel() < need or sq.data_ptr() != base.data_ptr():
            raise RuntimeError("fused norm: partial buffer layout")
        return base[:need]

    def _snapshot_norm(self, max_norm):
        # self.norm is one device word every step overwrites; callers that read a
        # step's norm later (training_utils._Pending reads step n after step n+1
        # is queued) need their own copy, queued on the same stream.
        if max_norm is not None:
            self.last_norm = self.norm.clone()

    def zero_grad(self, set_to_none=True):
        """The next backward overwrites the gradient arena (no memset; p.grad stays
        a view of the arena rather than becoming None)."""
        eng = self._engine if self._engine is not None else _find_engine(self.param_groups[0]["params"])
        if eng is not None:
            eng.zero_grad()
        else:
            super().zero_grad(set_to_none)

    # ------------------------------------------------------------ state io
    def _sync(self):
        eng = self._engine
        if eng is not None:
            eng.sync_pending()

    def state_dict(self):
        self._sync()
        if self._moments_stale:
            raise RuntimeError("sharded FusedAdam: call consolidate() on every rank before state_dict()")
        if self._engine is not None:
            for p in self.param_groups[0]["params"]:
                self.state[p]["step"] = torch.tensor(float(self._nstl_step))
        sd = super().state_dict()
        for s in sd["state"].values():
            for k, v in list(s.items()):
                if torch.is_tensor(v) and k != "step":
                    s[k] = v.clone()
        return sd

    def load_state_dict(self, state_dict):
        self._sync()
        super().load_state_dict(state_dict)
        params = self.param_groups[0]["params"]
        loaded = {p: dict(self.state[p]) for p in params if p in self.state}
        steps = [float(s["step"]) for s in loaded.values() if "step" in s]
        self._nstl_step = int(max(steps)) if steps else 0
        if self._engine is None and _find_engine(params) is None:
            return  # engine not built yet: keep torch-style state; bound on first step
        eng = self._bind()
        with torch.no_grad():
            for p in params:
                views = self._state_views(p)
                if p in loaded and "exp_avg" in loaded[p]:
                    views["exp_avg"].copy_(loaded[p]["exp_avg"].to(eng.device))
                    views["exp_avg_sq"].copy_(loaded[p]["exp_avg_sq"].to(eng.device))
                self.state[p] = views


def _find_engine(params):
    for p in params:
        eng = getattr(p, "_nstl_engine", None)
        if eng is not None:
            return eng()
    return None

