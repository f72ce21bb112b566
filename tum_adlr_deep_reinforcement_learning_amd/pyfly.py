"""PyFly-compatible facade over one engine handle.

``PyFly(config_path, parameter_path, config_kw)`` with ``seed``, ``reset(state,
turbulence_noise)``, ``step(commands) -> (success, info)`` and
``state[name].value`` -- the single-aircraft API of pyfly.py:1030-1448.  Unlike
the reference, the aircraft lives on the GPU: ``step`` launches the fused
kernel for this one lane (batch size ``num_aircraft``, default 1), and reading
``state[...]`` copies the SoA block back.  For throughput use :class:`Engine`
or :class:`FixedWingVecEnv` directly; this class exists so code written
against the reference's simulator runs unchanged.
"""
import numpy as np
import torch

from . import config as C
from .engine import Engine

_ODE_ROWS = {"omega_p": 4, "omega_q": 5, "omega_r": 6, "position_n": 7, "position_e": 8, "position_d": 9,
             "velocity_u": 10, "velocity_v": 11, "velocity_w": 12}
_DER_ROWS = {"roll": 0, "pitch": 1, "yaw": 2, "Va": 3, "alpha": 4, "beta": 5, "elevator": 6, "aileron": 7}


def energy_value(name, y, der, params, g):
    """EnergyVariable.calculate_value (pyfly.py:430-450) from a stored state: ODE state ``y`` [19],
    derived states ``der`` [8] (der[3] = Va), aircraft ``params`` (x8_param.mat names), gravity ``g``.

    The reference refreshes the energies only after a successful step (pyfly.py:1408-1411) and at
    reset.  Reading them from the device's stored state gives the same values after a failed step
    too: a failure leaves omega, position and Va at their pre-step values (stage conditioning fails
    before the save; at the save only the Euler-angle conditions can still fail, and they come
    before those variables are committed -- fw_device.hpp sim_step_masked)."""
    m, val = params["mass"], 0.0
    if name in ("energy_potential", "energy_total"):
        val += m * g * (-y[9])
    if name in ("energy_kinetic_rotational", "energy_kinetic", "energy_total"):
        for J, w in zip(("Jx", "Jy", "Jz"), y[4:7]):
            val += 0.5 * params[J] * w ** 2
    if name in ("energy_kinetic_translational", "energy_kinetic", "energy_total"):
        val += 0.5 * m * der[3] ** 2
    return val


class _VarView:
    """Read-only stand-in for pyfly's ``Variable`` (``.value``, ``.name``)."""

    def __init__(self, sim, name):
        self._sim, self.name = sim, name

    @property
    def value(self):
        return self._sim._value(self.name)

    def __repr__(self):
        return "%s: %r" % (self.name, self.value)


class SimulatorView:
    """``state[name].value`` access to aircraft ``index`` of an :class:`Engine` (pyfly.py:1054-1083 names)."""

    def __init__(self, engine, index=0):
        self.engine, self.index = engine, int(index)
        spec = engine.sim_spec
        self.dynamics = list(spec.dynamics)
        names = list(_ODE_ROWS) + list(_DER_ROWS) + ["attitude", "wind_n", "wind_e", "wind_d", "energy_potential",
                                                      "energy_kinetic", "energy_kinetic_rotational",
                                                      "energy_kinetic_translational", "energy_total"]
        names += self.dynamics
        self.state = {n: _VarView(self, n) for n in names}
        self._p = dict(zip(C.PARAM_NAMES, spec.struct().param))
        self._g = float(spec.struct().g)

    @property
    def cur_sim_step(self):
        s, _ = self.engine.steps()
        return int(s[self.index])

    def _block(self, blk):
        return self.engine.get_block(blk)[:, self.index].double().cpu().numpy()

    def _value(self, name):
        if name in _ODE_ROWS:
            return float(self._block(C.FW_BLK_ODE)[_ODE_ROWS[name]])
        if name in _DER_ROWS:
            return float(self._block(C.FW_BLK_DERIVED)[_DER_ROWS[name]])
        if name == "attitude":
            return self._block(C.FW_BLK_ODE)[0:4]
        if name in self.dynamics:
            return float(self._block(C.FW_BLK_ODE)[13 + self.dynamics.index(name)])
        if name.startswith("wind_"):
            # steady component; pyfly's wind_* also adds the current turbulence sample (pyfly.py:832-844)
            return float(self._block(C.FW_BLK_WIND)["ned".index(name[-1])])
        if name.startswith("energy"):
            return self._energy(name)
        raise KeyError(name)

    def _energy(self, name):
        return energy_value(name, self._block(C.FW_BLK_ODE), self._block(C.FW_BLK_DERIVED), self._p, self._g)

    def get_states_vector(self, states, attribute="value"):
        return [self.state[s].value for s in states]


class PyFly(SimulatorView):
    """Drop-in for ``pyfly.PyFly`` (pyfly.py:1030-1448) backed by the fused HIP step."""

    def __init__(self, config_path=None, parameter_path=None, config_kw=None, device=None, precision="float64",
                 num_aircraft=1):
        spec = C.build_sim(config_path, parameter_path, config_kw)
        self.cfg = spec.cfg
        self.dt = spec.struct().dt
        engine = Engine(spec, None, num_aircraft, device=device, precision=precision)
        super().__init__(engine, 0)
        self._cmd = torch.zeros(num_aircraft, 3, dtype=engine.dtype, device=engine.device)

    def seed(self, seed=None):
        """PyFly.seed (pyfly.py:1251-1260); aircraft i draws from Philox stream (seed, i)."""
        self.engine.seed(seed)

    def reset(self, state=None, turbulence_noise=None):
        """PyFly.reset (pyfly.py:1262-1311).  ``state`` is the reference's dict (NaN / missing = sample)."""
        n = self.engine.n
        self.engine.set_noise(turbulence_noise)  # Dryden.reset(noise): None draws fresh noise (dryden.py:174-188)
        init = C.init_array(state, n, self.engine.sim_spec) if state is not None else None
        self.engine.reset(init=init, want_obs=False)

    def step(self, commands):
        """PyFly.step (pyfly.py:1358-1420): returns ``(success, info)`` with ``info["termination"]`` on failure."""
        c = torch.as_tensor(np.asarray(commands, dtype=np.float64), dtype=self.engine.dtype)
        self._cmd.copy_(c.reshape(-1, 3).expand(self.engine.n, 3))
        success, term = self.engine.sim_step(self._cmd)
        ok = bool(success[self.index].item())
        if ok:
            return True, {}
        from .vec_env import termination_name
        return False, {"termination": termination_name(term[self.index].item(), tuple(self.dynamics))}
