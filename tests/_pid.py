"""PI/PID attitude + airspeed controller used to drive deterministic parity
scenarios -- restated from the reference's test driver
magpie/libs/pyfly/pyfly/pid_controller.py:4-109 (gains and limits)."""
import numpy as np


class PID:
    def __init__(self, phi_r, theta_r, va_r, dt=0.01):
        self.dt = dt
        self.set_reference(phi_r, theta_r, va_r)
        self.int_va = self.int_roll = self.int_pitch = 0.0

    def set_reference(self, phi, theta, va):
        self.phi_r, self.theta_r, self.va_r = phi, theta, va

    def action(self, obs):
        """obs in the default layout: roll, pitch, Va, p, q, r, ..."""
        phi, theta, va, p, q = obs[0], obs[1], obs[2], obs[3], obs[4]
        e_v, e_phi, e_th = va - self.va_r, phi - self.phi_r, theta - self.theta_r
        self.int_va += self.dt * e_v
        self.int_roll += self.dt * e_phi
        self.int_pitch += self.dt * e_th
        d_t = 0 - 0.5 * e_v - 0.1 * self.int_va
        d_a = -1 * e_phi - 0 * self.int_roll - 0.5 * p
        d_e = 0 - (-4) * e_th - (-0.75) * self.int_pitch - (-0.1) * q
        return np.array([np.clip(d_e, np.radians(-30), np.radians(35)), np.clip(d_a, np.radians(-30), np.radians(30)),
                         np.clip(d_t, 0, 1.0)])
