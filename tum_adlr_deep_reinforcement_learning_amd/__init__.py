"""MI355X-native batched fixed-wing flight-dynamics stepper.

Drop-in for the PyFly.step() / FixedWingAircraft.step() / SB3 VecEnv hot path of
MoritzSchueler96/TUM_ADLR_Deep_Reinforcement_Learning ("magpie").  The physics
and env epilogue run as one fused HIP kernel for gfx950 (csrc/), reached
through the C ABI declared in include/fwsim.h (libfwsim.so).
"""
__version__ = "0.1.0"
