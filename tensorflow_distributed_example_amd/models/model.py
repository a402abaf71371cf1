"""Keras ``Sequential`` model: build / summary / compile / fit / evaluate /
predict / weights I/O (distributed_with_keras.py:33-43,
mnist_keras_distributed.py:79-117).

Variables are created under the current distribution strategy (``strategy.scope()``,
distributed_with_keras.py:51) on its first local device and replicated per
replica at the first fit/evaluate (MirroredVariable semantics; chief broadcast).
"""
from __future__ import annotations

import json
from typing import Optional

import numpy as np
import torch

from .. import backend as K
from .. import losses as LS
from .. import metrics as MT
from .. import optimizers as OP
from ..parallel import strategy as DS
from ..train import engine as E
from ..train import params as P
from ..train import runner as RN
from . import layers as L


class _SingleReplica(DS.Strategy):
    def __init__(self, device):
        super().__init__([device], DS.CM.NullCommunicator(), name="single")


class Model:
    def __new__(cls, *args, **kw):
        # keras.Model(inputs, outputs) builds a functional (DAG) model
        if cls is Model and (len(args) >= 2 or "inputs" in kw or "outputs" in kw):
            return object.__new__(Functional)
        return object.__new__(cls)

    def __init__(self, name: Optional[str] = None):
        self.name = name or K.unique_name(self._prefix)
        self._store: Optional[P.ParamStore] = None
        self._strategy = None
        self._stores = {}
        self._programs = {}
        self.optimizer = None
        self.loss = None
        self.compiled_metrics = []
        self._metric_names = []
        self.steps_per_execution = 1
        self.history = None
        self.stop_training = False

    # ------------------------------------------------------------------ variables
    @property
    def built(self):
        return self._store is not None

    def _nodes(self):
        """Execution graph: [(layer, input tensor ids, output tensor id)] in topological order;
        tensor 0 is the model input, the last node's output is the model output."""
        raise NotImplementedError

    def _create_store(self):
        st = DS.get_strategy()
        self._strategy = st
        specs = [s for layer in self.layers for s in layer.weight_specs]
        for layer in self.layers:
            layer._model = self
        self._store = P.ParamStore(specs, st.local_devices[0], init=True, generator=K.make_generator(0))

    def _replica_stores(self, strategy):
        if isinstance(strategy, _SingleReplica):
            return [self._primary_store()]
        key = id(strategy)
        if key not in self._stores:
            if self._store.device != strategy.local_devices[0]:
                self._store = self._store.clone_to(strategy.local_devices[0])
            self._stores = {key: strategy.replicate_store(self._store)}
            self._programs = {}
        return self._stores[key]

    def _primary_store(self):
        return self._store

    def _all_stores(self):
        out = [self._store]
        for lst in self._stores.values():
            out += [s for s in lst if s is not self._store]
        return out

    def _program(self, kind, global_batch, single_replica=False):
        strategy = _SingleReplica(self._store.device) if single_replica else self._strategy
        key = (kind, int(global_batch), id(strategy) if not single_replica else "single",
               self.steps_per_execution if kind == "train" else 1)
        prog = self._programs.get(key)
        if prog is None:
            if kind == "train" and self.optimizer is None:
                raise RuntimeError("You must compile your model before training/testing.")
            prog = RN.Program(self, strategy, global_batch, training=(kind == "train"),
                              steps_per_execution=self.steps_per_execution)
            self._programs[key] = prog
        return prog

    def _set_iterations(self, step: int):
        """Restore the optimizer step counter (host and every plan's device counter)."""
        if self.optimizer is not None:
            self.optimizer.iterations = int(step)
        for prog in self._programs.values():
            for plan in prog.plans:
                plan.iterations.fill_(int(step))

    def _weights_changed(self):
        """Propagate replica-0 values to every replica and refresh kernel caches."""
        st = self._strategy
        lst = self._stores.get(id(st))
        if lst:
            st.broadcast_stores(lst)
        for prog in self._programs.values():
            prog.on_weights_loaded()

    def _sync_on_read(self):
        """MEAN of the SyncOnRead (BN moving-stat) variables across replicas (C4)."""
        st = self._strategy
        lst = self._stores.get(id(st)) if st is not None else None
        has_state = any(not seg.trainable for seg in self._store.segments.values())
        if not lst or st.num_replicas_in_sync == 1 or not has_state:
            return self._store.state.detach().clone()
        bufs = [s.state.clone() for s in lst]
        st.comm.all_reduce_(bufs, op="mean")
        st._sync_all(lst)
        return bufs[0]

    # ------------------------------------------------------------------ weights API
    def _spec_list(self):
        return [s for layer in self.layers for s in layer.weight_specs]

    @property
    def weights(self):
        return [self._store.view(s.full_name) for s in self._spec_list()]

    @property
    def trainable_weights(self):
        return [self._store.view(s.full_name) for s in self._spec_list() if s.trainable]

    @property
    def non_trainable_weights(self):
        return [self._store.view(s.full_name) for s in self._spec_list() if not s.trainable]

    @property
    def variables(self):
        return self.weights

    def variable_names(self):
        return [s.full_name for s in self._spec_list()]

    def get_weights(self):
        self._require_built()
        state = self._sync_on_read()
        out = []
        for s in self._spec_list():
            seg = self._store.segments[s.full_name]
            if seg.trainable:
                out.append(self._store.view(s.full_name).detach().cpu().numpy().copy())
            else:
                out.append(state[seg.offset: seg.offset + seg.numel].view(seg.shape).cpu().numpy().copy())
        return out

    def set_weights(self, weights):
        self._require_built()
        specs = self._spec_list()
        if len(weights) != len(specs):
            raise ValueError(f"expected {len(specs)} arrays, got {len(weights)}")
        self._store.load_dict({s.full_name: w for s, w in zip(specs, weights)})
        self._weights_changed()

    def state_dict(self):
        self._require_built()
        state = self._sync_on_read()
        out = {}
        for n in self._store.order:
            seg = self._store.segments[n]
            if seg.trainable:
                out[n] = self._store.view(n).detach().cpu().clone()
            else:
                out[n] = state[seg.offset: seg.offset + seg.numel].view(seg.shape).cpu().clone()
        return out

    def load_state_dict(self, d, strict=True):
        self._store.load_dict(d, strict=strict)
        self._weights_changed()

    def save_weights(self, filepath, overwrite=True, save_format=None):
        from ..io import checkpoint as CK
        CK.save_model_weights(self, filepath, save_format)

    def load_weights(self, filepath):
        from ..io import checkpoint as CK
        CK.load_model_weights(self, filepath)

    def _require_built(self):
        if not self.built:
            raise ValueError(f"model {self.name} is not built yet; give the first layer an input_shape "
                             "or call build()")

    def count_params(self):
        return int(sum(l.count_params() for l in self.layers))

    # ------------------------------------------------------------------ compile/fit
    def compile(self, optimizer="rmsprop", loss=None, metrics=None, loss_weights=None, weighted_metrics=None,
                run_eagerly=None, steps_per_execution=None, jit_compile=None, **kw):
        self._require_built()
        self.optimizer = OP.get(optimizer if optimizer != "rmsprop" else "sgd")
        self.loss = LS.get(loss)
        self.compiled_metrics = list(metrics or [])
        self._metric_names = MT.resolve(metrics)
        if steps_per_execution is not None:
            self.steps_per_execution = int(steps_per_execution)
        if DS.has_strategy():
            st = DS.get_strategy()
            if st is not self._strategy:
                self._strategy = st
        elif self._strategy is None:
            self._strategy = DS.get_strategy()
        self._programs = {}

    def fit(self, x=None, y=None, batch_size=None, epochs=1, verbose="auto", callbacks=None, validation_data=None,
            steps_per_epoch=None, initial_epoch=0, shuffle=True, validation_steps=None, validation_freq=1, **kw):
        return E.fit(self, x, y, batch_size, epochs, verbose, callbacks, validation_data, steps_per_epoch,
                     initial_epoch, shuffle, validation_steps, validation_freq)

    def evaluate(self, x=None, y=None, batch_size=None, verbose="auto", steps=None, return_dict=False, **kw):
        return E.evaluate(self, x, y, batch_size, verbose, steps, return_dict)

    def predict(self, x, batch_size=None, verbose=0, steps=None, **kw):
        return E.predict(self, x, batch_size, verbose, steps)

    # ------------------------------------------------------------------ direct call (reference ops)
    def __call__(self, x, training=False):
        self._require_built()
        from ..train.program import ReferencePlan
        plan = ReferencePlan(self, self._store, self._store.device, 1, 1, None, self.loss or LS.SparseCategoricalCrossentropy())
        x = torch.as_tensor(np.asarray(x) if not torch.is_tensor(x) else x, device=self._store.device).float()
        x = x.reshape((x.shape[0],) + tuple(self.input_shape[1:]))
        plan.strip_softmax = False
        with torch.no_grad():
            return plan._forward(x, plan._weights(None), training)


class Sequential(Model):
    _prefix = "sequential"

    def __init__(self, layers=None, name=None):
        super().__init__(name)
        self._layers: list = []
        self._input_shape = None
        for l in layers or []:
            self.add(l)

    @property
    def layers(self):
        return [l for l in self._layers if not isinstance(l, L.InputLayer)]

    def _nodes(self):
        return [(l, [i], i + 1) for i, l in enumerate(self.layers)]

    def add(self, layer):
        if self.built:
            raise RuntimeError("cannot add layers to a built model")
        if not isinstance(layer, L.Layer):
            raise TypeError(f"expected a Layer, got {layer!r}")
        self._layers.append(layer)
        if len(self._layers) == 1 and layer.input_shape_arg is not None:
            self._input_shape = layer.input_shape_arg
        if self._input_shape is not None:
            self._build_shapes()
            if all(l.built for l in self._layers):
                pass

    def _build_shapes(self):
        s = tuple(self._input_shape)
        for l in self._layers:
            s = l._build_shapes(s)
        self._output_shape = s

    def build(self, input_shape=None):
        if input_shape is not None:
            self._input_shape = tuple(input_shape[1:]) if len(input_shape) > 1 and input_shape[0] is None \
                else tuple(input_shape)
        if self._input_shape is None:
            raise ValueError("input shape unknown")
        self._build_shapes()
        if self._store is None:
            self._create_store()

    def _ensure_store(self):
        if self._store is None and self._input_shape is not None:
            self._build_shapes()
            self._create_store()

    @property
    def built(self):
        return self._store is not None

    def _require_built(self):
        self._ensure_store()
        super()._require_built()

    @property
    def input_shape(self):
        return (None,) + tuple(self._input_shape)

    @property
    def output_shape(self):
        return (None,) + tuple(self._output_shape)

    def summary(self, line_length=65, positions=None, print_fn=None):
        self._require_built()
        pf = print_fn or print
        pos = positions or [0.45, 0.85, 1.0]
        pos = [int(line_length * p) for p in pos]

        def row(fields):
            line = ""
            for i, f in enumerate(fields):
                if i:
                    line = line[:pos[i - 1] - 1] + " "
                line += str(f)
                line = line[:pos[i]].ljust(pos[i])
            return line

        pf(f'Model: "{self.name}"')
        pf("_" * line_length)
        pf(row([" Layer (type)", "Output Shape", "Param #"]))
        pf("=" * line_length)
        for i, l in enumerate(self.layers):
            pf(row([f" {l.name} ({type(l).__name__})", str((None,) + tuple(l.output_shape)).replace(",)", ",)"),
                    str(l.count_params())]))
            if i != len(self.layers) - 1:
                pf("")
        pf("=" * line_length)
        tot = self.count_params()
        tr = sum(int(np.prod(s.shape)) for s in self._spec_list() if s.trainable)
        pf(f"Total params: {tot:,}")
        pf(f"Trainable params: {tr:,}")
        pf(f"Non-trainable params: {tot - tr:,}")
        pf("_" * line_length)

    def get_config(self):
        return {"name": self.name, "layers": [{"class_name": type(l).__name__, "config": l.get_config()}
                                              for l in self._layers],
                "input_shape": list(self._input_shape) if self._input_shape else None}

    def to_json(self):
        return json.dumps({"class_name": "Sequential", "config": self.get_config()})

    @classmethod
    def from_config(cls, cfg, keep_names=True):
        m = cls(name=cfg.get("name") if keep_names else None)
        first = True
        for lc in cfg["layers"]:
            c = dict(lc["config"])
            if not keep_names:
                c.pop("name", None)
            if first and cfg.get("input_shape"):
                c["input_shape"] = tuple(cfg["input_shape"])
            first = False
            m.add(L.from_config(lc["class_name"], c))
        return m


class Functional(Model):
    """Functional-API model: ``Model(inputs=Input(...), outputs=...)`` over a DAG of layer
    calls (multi-consumer tensors, ``Add`` joins) — used by the ResNet-18 stress config."""
    _prefix = "model"

    def __init__(self, inputs=None, outputs=None, name=None):
        super().__init__(name)
        if isinstance(inputs, (list, tuple)):
            if len(inputs) != 1:
                raise ValueError("only single-input models are supported")
            inputs = inputs[0]
        if isinstance(outputs, (list, tuple)):
            if len(outputs) != 1:
                raise ValueError("only single-output models are supported")
            outputs = outputs[0]
        self._input = inputs
        self._output = outputs
        order, seen = [], set()

        def visit(t):
            if id(t) in seen:
                return
            seen.add(id(t))
            for u in t.inputs:
                visit(u)
            order.append(t)

        visit(outputs)
        if inputs not in order:
            raise ValueError("outputs are not connected to inputs")
        ids = {id(inputs): 0}
        self._graph = []
        for t in order:
            if t is inputs:
                continue
            if t.producer is None:
                raise ValueError(f"disconnected input {t}")
            ids[id(t)] = len(ids)
            self._graph.append((t.producer, [ids[id(u)] for u in t.inputs], ids[id(t)]))
        used = [l for l, _, _ in self._graph]
        if len(set(map(id, used))) != len(used):
            raise ValueError("a layer is called more than once (shared layers are not supported)")
        self._input_shape = tuple(inputs.shape[1:])
        self._output_shape = tuple(outputs.shape[1:])

    @property
    def layers(self):
        return [l for l, _, _ in self._graph]

    def _nodes(self):
        return list(self._graph)

    def build(self, input_shape=None):
        if self._store is None:
            self._create_store()

    @property
    def built(self):
        return self._store is not None

    def _require_built(self):
        if self._store is None:
            self._create_store()

    @property
    def input_shape(self):
        return (None,) + tuple(self._input_shape)

    @property
    def output_shape(self):
        return (None,) + tuple(self._output_shape)

    def summary(self, line_length=98, print_fn=None):
        self._require_built()
        pf = print_fn or print
        producers = {0: "input"}
        for l, _, o in self._graph:
            producers[o] = l.name
        pf(f'Model: "{self.name}"')
        pf("_" * line_length)
        pf(f"{' Layer (type)':<34}{'Output Shape':<24}{'Param #':<10}Connected to")
        pf("=" * line_length)
        for l, ins, _ in self._graph:
            pf(f"{(' ' + l.name + ' (' + type(l).__name__ + ')')[:33]:<34}"
               f"{str((None,) + tuple(l.output_shape)):<24}{l.count_params():<10}"
               f"{', '.join(producers[i] for i in ins)}")
        pf("=" * line_length)
        tot = self.count_params()
        tr = sum(int(np.prod(s.shape)) for s in self._spec_list() if s.trainable)
        pf(f"Total params: {tot:,}")
        pf(f"Trainable params: {tr:,}")
        pf(f"Non-trainable params: {tot - tr:,}")
        pf("_" * line_length)

    def get_config(self):
        return {"name": self.name, "input_shape": list(self._input_shape),
                "layers": [{"class_name": type(l).__name__, "config": l.get_config(), "inbound": ins}
                           for l, ins, _ in self._graph]}

    def to_json(self):
        return json.dumps({"class_name": "Functional", "config": self.get_config()})

    @classmethod
    def from_config(cls, cfg, keep_names=True):
        t = {0: L.Input(tuple(cfg["input_shape"]))}
        for i, lc in enumerate(cfg["layers"]):
            c = dict(lc["config"])
            if not keep_names:
                c.pop("name", None)
            layer = L.from_config(lc["class_name"], c)
            ins = [t[j] for j in lc["inbound"]]
            t[i + 1] = layer(ins if layer.multi_input else ins[0])
        return cls(t[0], t[len(cfg["layers"])], name=cfg.get("name") if keep_names else None)
