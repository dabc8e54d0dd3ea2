"""ctypes binding of the VRACER agent's C-ABI (include/korali_amd.h, kg_vracer_*).

The device path of Korali's `Agent / Continuous / VRACER` solver
(solver/agent/agent.cpp.base, continuous/VRACER/VRACER.cpp.base) with the
continuous Normal policy and the CartPole environment of
examples/learning/reinforcement/cartpole.  Every call goes to the HIP
kernels of korali_amd/libkorali_amd.so; there is no CPU fallback.
"""
import ctypes as C

import numpy as np

from .native import KoraliDeviceError, check, lib

# replay-memory / agent fields with a non-float32 element type
_DTYPES = {
    "environment_id": np.int32, "termination": np.int32, "on_policy": np.int32, "episode_pos": np.int32,
    "env_steps": np.int32, "env_ids": np.int32, "finished_env": np.int32, "mini_batch": np.uint32,
    "episode_id": np.int64, "env_u": np.float64, "env_sample_ids": np.uint64, "reward_rescaling_count": np.int64, "meta_phase_ticks": np.uint64,
}


class _VracerCfg(C.Structure):
    _fields_ = [
        ("state_size", C.c_size_t), ("action_size", C.c_size_t), ("hidden_size", C.c_size_t),
        ("hidden_layers", C.c_size_t), ("environments", C.c_size_t), ("environment_count", C.c_size_t),
        ("mini_batch_size", C.c_size_t), ("replay_maximum_size", C.c_size_t), ("replay_start_size", C.c_size_t),
        ("max_episode_steps", C.c_size_t), ("experiences_between_policy_updates", C.c_double),
        ("discount_factor", C.c_double), ("learning_rate", C.c_double),
        ("importance_weight_truncation_level", C.c_double), ("off_policy_cutoff_scale", C.c_double),
        ("off_policy_target", C.c_double), ("off_policy_annealing_rate", C.c_double),
        ("off_policy_refer_beta", C.c_double), ("l2_regularization_enabled", C.c_int),
        ("l2_regularization_importance", C.c_double), ("initial_exploration_noise", C.POINTER(C.c_double)),
        ("seed", C.c_uint64), ("device", C.c_int), ("policy_distribution", C.c_int),
        ("action_lower_bounds", C.POINTER(C.c_double)), ("action_upper_bounds", C.POINTER(C.c_double)),
        ("reward_rescaling", C.c_int), ("state_rescaling", C.c_int), ("host_environment", C.c_int),
    ]


_BOUND = False


def _lib():
    global _BOUND
    L = lib()
    if not _BOUND:
        vp, sz, cp = C.c_void_p, C.c_size_t, C.c_char_p
        fp = C.POINTER(C.c_float)
        L.kg_vracer_create.argtypes = [C.POINTER(_VracerCfg), C.POINTER(vp)]
        for f in ("kg_vracer_destroy", "kg_vracer_synchronize"):
            getattr(L, f).argtypes = [vp]
        L.kg_vracer_hyperparameter_count.argtypes = [vp, C.POINTER(sz)]
        L.kg_vracer_field_size.argtypes = [vp, cp, C.POINTER(sz), C.POINTER(sz)]
        L.kg_vracer_get_field.argtypes = [vp, cp, vp, sz]
        L.kg_vracer_set_field.argtypes = [vp, cp, vp, sz]
        L.kg_vracer_get_scalar.argtypes = [vp, cp, C.POINTER(C.c_double)]
        L.kg_vracer_set_scalar.argtypes = [vp, cp, C.c_double]
        L.kg_vracer_run_policy.argtypes = [vp, fp, sz, fp]
        L.kg_vracer_set_action_noise.argtypes = [vp, fp, sz]
        L.kg_vracer_environment_step.argtypes = [vp, C.POINTER(sz)]
        L.kg_vracer_save_state.argtypes = [vp, cp, vp, sz]
        L.kg_vracer_load_state.argtypes = [vp, cp, vp, sz, C.POINTER(sz)]
        L.kg_vracer_train_policy.argtypes = [vp, sz]
        L.kg_vracer_train_policy_minibatch.argtypes = [vp, C.POINTER(C.c_uint32), sz]
        L.kg_vracer_training_step.argtypes = [vp, C.POINTER(sz), C.POINTER(sz)]
        L.kg_vracer_rescale_states.argtypes = [vp]
        L.kg_vracer_train_pending.argtypes = [vp, C.POINTER(sz)]
        ip = C.POINTER(C.c_int)
        L.kg_vracer_host_launch.argtypes = [vp, fp, ip]
        L.kg_vracer_host_act.argtypes = [vp, fp]
        L.kg_vracer_host_feed.argtypes = [vp, fp, fp, ip, fp, ip, C.POINTER(sz)]
        u64p = C.POINTER(C.c_uint64)
        L.kg_vracer_test_episodes.argtypes = [vp, u64p, u64p, sz, fp]
        L.kg_vracer_stream.argtypes = [vp, C.POINTER(vp)]
        L.kg_vracer_profile.argtypes = [vp, C.c_int]
        L.kg_vracer_profile_read.argtypes = [vp, cp, C.POINTER(C.c_double), C.POINTER(sz)]
        _BOUND = True
    return L


def _fptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


class VracerDevice:
    """One VRACER agent on one GPU.  Keyword names follow the reference's JSON
    keys (agent.config / VRACER.config), e.g. `mini_batch_size` = "Mini Batch"/"Size"."""

    def __init__(self, state_size=4, action_size=1, hidden_size=256, hidden_layers=2, environments=4096,
                 environment_count=3, mini_batch_size=256, replay_maximum_size=262144, replay_start_size=131072,
                 max_episode_steps=500, experiences_between_policy_updates=1.0, discount_factor=0.995,
                 learning_rate=1e-4, importance_weight_truncation_level=1.0, off_policy_cutoff_scale=4.0,
                 off_policy_target=0.1, off_policy_annealing_rate=0.0, off_policy_refer_beta=0.3,
                 l2_regularization_enabled=False, l2_regularization_importance=1e-4, initial_exploration_noise=1.0,
                 seed=0, device=0, hyperparameters=None, policy_distribution="Normal", action_lower_bound=-np.inf,
                 action_upper_bound=np.inf, reward_rescaling=False, state_rescaling=False, host_environment=False):
        L = _lib()
        self.S, self.A, self.H, self.L = state_size, action_size, hidden_size, hidden_layers
        self.E, self.B, self.O = environments, mini_batch_size, 1 + 2 * action_size
        noise = np.ascontiguousarray(np.broadcast_to(np.asarray(initial_exploration_noise, np.float64),
                                                     (action_size,)))
        self._noise = noise
        pol = {"normal": 0, "clippednormal": 1}.get(policy_distribution.replace(" ", "").lower())
        if pol is None:
            raise KoraliDeviceError(f"Policy Distribution '{policy_distribution}' is not supported on the device")
        self._lb = np.ascontiguousarray(np.broadcast_to(np.asarray(action_lower_bound, np.float64), (action_size,)))
        self._ub = np.ascontiguousarray(np.broadcast_to(np.asarray(action_upper_bound, np.float64), (action_size,)))
        cfg = _VracerCfg(state_size, action_size, hidden_size, hidden_layers, environments, environment_count,
                         mini_batch_size, replay_maximum_size, replay_start_size, max_episode_steps,
                         experiences_between_policy_updates, discount_factor, learning_rate,
                         importance_weight_truncation_level, off_policy_cutoff_scale, off_policy_target,
                         off_policy_annealing_rate, off_policy_refer_beta, int(bool(l2_regularization_enabled)),
                         l2_regularization_importance, noise.ctypes.data_as(C.POINTER(C.c_double)), seed, device,
                         pol, self._lb.ctypes.data_as(C.POINTER(C.c_double)),
                         self._ub.ctypes.data_as(C.POINTER(C.c_double)), int(bool(reward_rescaling)),
                         int(bool(state_rescaling)), int(bool(host_environment)))
        h = C.c_void_p()
        check(L.kg_vracer_create(C.byref(cfg), C.byref(h)))
        self._h = h
        n = C.c_size_t()
        check(L.kg_vracer_hyperparameter_count(h, C.byref(n)))
        self.hyperparameter_count = n.value
        if hyperparameters is not None:
            self.set("hyperparameters", hyperparameters)

    def close(self):
        if getattr(self, "_h", None):
            _lib().kg_vracer_destroy(self._h)
            self._h = None

    __del__ = close

    # ---- fields and scalars
    def field_size(self, name):
        e, c = C.c_size_t(), C.c_size_t()
        check(_lib().kg_vracer_field_size(self._h, name.encode(), C.byref(e), C.byref(c)))
        return e.value, c.value

    def get(self, name, count=None):
        _, n = self.field_size(name)
        a = np.empty(n if count is None else count, _DTYPES.get(name, np.float32))
        check(_lib().kg_vracer_get_field(self._h, name.encode(), a.ctypes.data_as(C.c_void_p), a.nbytes))
        return a

    def set(self, name, values):
        a = np.ascontiguousarray(values, dtype=_DTYPES.get(name, np.float32)).ravel()
        check(_lib().kg_vracer_set_field(self._h, name.encode(), a.ctypes.data_as(C.c_void_p), a.nbytes))

    def scalar(self, name):
        v = C.c_double()
        check(_lib().kg_vracer_get_scalar(self._h, name.encode(), C.byref(v)))
        return v.value

    def set_scalar(self, name, value):
        check(_lib().kg_vracer_set_scalar(self._h, name.encode(), float(value)))

    @property
    def hyperparameters(self):
        return self.get("hyperparameters")

    # ---- agent operations
    def run_policy(self, states):
        X = np.ascontiguousarray(states, np.float32).reshape(-1, self.S)
        out = np.empty((X.shape[0], self.O), np.float32)
        check(_lib().kg_vracer_run_policy(self._h, _fptr(X), X.shape[0], _fptr(out)))
        return out

    def environment_step(self, noise=None):
        if noise is not None:
            z = np.ascontiguousarray(noise, np.float32).ravel()
            check(_lib().kg_vracer_set_action_noise(self._h, _fptr(z), z.size))
        n = C.c_size_t()
        check(_lib().kg_vracer_environment_step(self._h, C.byref(n)))
        return n.value

    def train_policy(self, updates=1):
        check(_lib().kg_vracer_train_policy(self._h, updates))

    def train_minibatch(self, ids):
        a = np.ascontiguousarray(ids, np.uint32)
        check(_lib().kg_vracer_train_policy_minibatch(self._h, a.ctypes.data_as(C.POINTER(C.c_uint32)), a.size))

    def training_step(self):
        n, u = C.c_size_t(), C.c_size_t()
        check(_lib().kg_vracer_training_step(self._h, C.byref(n), C.byref(u)))
        return n.value, u.value

    def rescale_states(self):
        """Agent::rescaleStates (training_step calls it where the reference does)"""
        check(_lib().kg_vracer_rescale_states(self._h))

    def test_episodes(self, sample_ids, launch_ids=None):
        """Testing episodes (Agent::testingGeneration): the cumulative reward of
        one deterministic CartPole episode per sample id."""
        sid = np.ascontiguousarray(sample_ids, np.uint64)
        lid = np.ascontiguousarray(np.arange(sid.size) if launch_ids is None else launch_ids, np.uint64)
        out = np.empty(sid.size, np.float32)
        u64p = C.POINTER(C.c_uint64)
        check(_lib().kg_vracer_test_episodes(self._h, sid.ctypes.data_as(u64p), lid.ctypes.data_as(u64p), sid.size,
                                             _fptr(out)))
        return out

    def synchronize(self):
        check(_lib().kg_vracer_synchronize(self._h))

    def save_state(self, path):
        """The whole training state (kg_vracer_save_state)."""
        check(_lib().kg_vracer_save_state(self._h, str(path).encode(), None, 0))

    def load_state(self, path):
        """Continue the run saved in `path` (same configuration)."""
        n = C.c_size_t(0)
        check(_lib().kg_vracer_load_state(self._h, str(path).encode(), None, 0, C.byref(n)))

    def profile(self, enable=True):
        check(_lib().kg_vracer_profile(self._h, int(bool(enable))))

    def profile_read(self, stage):
        ms, n = C.c_double(), C.c_size_t()
        check(_lib().kg_vracer_profile_read(self._h, stage.encode(), C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def stream(self):
        s = C.c_void_p()
        check(_lib().kg_vracer_stream(self._h, C.byref(s)))
        return s.value


__all__ = ["VracerDevice", "KoraliDeviceError"]
