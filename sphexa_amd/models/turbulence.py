"""Driven turbulence: stirring modes, Ornstein-Uhlenbeck phases and the VE propagator that adds the stirring force.

Parity (reference sph/include/sph/hydro_turb/):
  turbulence_data.hpp:40-170  TurbulenceData: decayTime = L/(2 v), variance = sqrt(E/decayTime),
                              solWeightNorm, N(0, variance) initial phases, state saved as "turbulence::*" step
                              attributes plus the RNG state ("rngEngineState")
  create_modes.hpp:40-210     createStirringModes: parabolic (spectForm 1) / band (0) spectra on the integer k lattice
                              with the (kx, +-ky, +-kz) mirror modes, power-law random modes (2)
  phases.hpp:40-70            computePhases: Helmholtz projection with solenoidal weight
  driver.hpp:40-90            updateNoise (OU update) + computeStirring
  main/src/propagator/turb_ve.hpp:52-103  TurbVeProp
The per-particle stirring sum runs in ``_sphx_hip.compute_stirring`` (mode table staged in LDS) on the GPU.
The RNG reproduces std::mt19937 with libstdc++'s uniform/normal distributions bit for bit (utils/std_random.py), and
"rngEngineState" is the engine's text serialization stored as a char array, as in the reference.
"""

from __future__ import annotations

import math
import sys

import numpy as np
import torch

from ..ops import _lib
from ..utils.std_random import StdMt19937
from .propagators import HydroVeProp


def create_stirring_modes(L, st_max_modes, stir_max, stir_min, spect_form, power_law_exp, angles_exp, rng,
                          ndim=3):
    """returns (modes [M,3], amplitudes [M])"""
    twopi = 2.0 * math.pi
    kc = 0.5 * (stir_min + stir_max) if spect_form == 1 else stir_min
    modes, amps = [], []
    if spect_form != 2:
        parab = -4.0 / ((stir_max - stir_min) ** 2)
        ik = np.arange(0, 257)
        kk = twopi * ik / L
        KX, KY, KZ = np.meshgrid(kk, kk, kk, indexing="ij")
        K = np.sqrt(KX ** 2 + KY ** 2 + KZ ** 2)
        sel = np.argwhere((K >= stir_min) & (K <= stir_max))  # lexicographic ikx, iky, ikz order
        for a, b, c in sel:
            if len(modes) + 4 > st_max_modes:
                print("Too many stirring modes", file=sys.stderr)
                break
            kx, ky, kz, k = kk[a], kk[b], kk[c], K[a, b, c]
            amp = 1.0
            if spect_form == 1:
                amp = abs(parab * (k - kc) ** 2 + 1.0)
            amp = 2.0 * math.sqrt(amp) * (kc / k) ** (0.5 * (ndim - 1))
            for sy, sz in ((1, 1), (-1, 1), (1, -1), (-1, -1)):
                modes.append((kx, sy * ky, sz * kz))
                amps.append(amp)
    else:
        ikmin = max(1, int(stir_min * L / twopi + 0.5))
        ikmax = int(stir_max * L / twopi + 0.5)
        for ik in range(ikmin, ikmax + 1):
            nang = int(2 ** ndim * math.ceil(ik ** angles_exp))
            for _ in range(nang):
                phi = twopi * rng.uniform()
                theta = math.acos(1.0 - 2.0 * rng.uniform())
                rand = ik + rng.uniform() - 0.5
                kx = twopi * round(rand * math.sin(theta) * math.cos(phi)) / L
                ky = twopi * round(rand * math.sin(theta) * math.sin(phi)) / L
                kz = twopi * round(rand * math.cos(theta)) / L
                k = math.sqrt(kx * kx + ky * ky + kz * kz)
                if stir_min <= k <= stir_max:
                    if len(modes) + 4 > st_max_modes:
                        break
                    amp = (k / kc) ** power_law_exp
                    amp = math.sqrt(amp * (ik ** (ndim - 1) * 4.0 * math.sqrt(3.0) / nang)) * (kc / k) ** ((ndim - 1) / 2)
                    modes.append((kx, ky, kz))
                    amps.append(amp)
    return np.asarray(modes, dtype=np.float64).reshape(-1, 3), np.asarray(amps, dtype=np.float64)


def compute_phases(modes, ou_phases, sol_weight):
    """Helmholtz decomposition of the OU phases: returns (real [M,3], imag [M,3])"""
    P = ou_phases.reshape(-1, 3, 2)
    kk = (modes * modes).sum(1)
    ka = (modes * P[:, :, 1]).sum(1)
    kb = (modes * P[:, :, 0]).sum(1)
    diva = modes * (ka / kk)[:, None]
    divb = modes * (kb / kk)[:, None]
    curla = P[:, :, 0] - divb
    curlb = P[:, :, 1] - diva
    re = sol_weight * curla + (1.0 - sol_weight) * divb
    im = sol_weight * curlb + (1.0 - sol_weight) * diva
    return re, im


class TurbulenceData:
    PREFIX = "turbulence::"

    def __init__(self, constants, verbose=False):
        self.sol_weight = float(constants["solWeight"])
        self.rng = StdMt19937(int(constants["rngSeed"]))
        eps = float(constants["epsilon"])
        L = float(constants["Lbox"])
        vel = float(constants["stMachVelocity"])
        energy = float(constants["stEnergyPrefac"]) * vel ** 3 / L
        twopi = 2 * math.pi
        self.decay_time = L / (2.0 * vel)
        self.variance = math.sqrt(energy / self.decay_time)
        ndim = 3
        self.sol_weight_norm = (math.sqrt(3.0) * math.sqrt(3.0 / ndim) /
                                math.sqrt(1.0 - 2.0 * self.sol_weight + ndim * self.sol_weight ** 2))
        self.modes, self.amplitudes = create_stirring_modes(
            L, int(constants["stMaxModes"]), (3.0 + eps) * twopi / L, (1.0 - eps) * twopi / L,
            int(constants["stSpectForm"]), float(constants["powerLawExp"]), float(constants["anglesExp"]), self.rng)
        if verbose:
            print(f"Total Number of Stirring Modes: {self.num_modes}")
        self.phases = self.rng.normal(6 * self.num_modes, 0.0, self.variance)
        self._dev_table = None

    @property
    def num_modes(self):
        return self.modes.shape[0]

    def update_noise(self, dt):
        a = math.exp(-dt / self.decay_time)
        b = math.sqrt(1.0 - a * a)
        self.phases = self.phases * a + self.variance * b * self.rng.normal(self.phases.size)

    def mode_table(self):
        """[M, 10] float32 table {kx, ky, kz, 0, amp*Re(3), amp*Im(3)} for the GPU kernel"""
        re, im = compute_phases(self.modes, self.phases, self.sol_weight)
        t = np.zeros((self.num_modes, 10), dtype=np.float32)
        t[:, 0:3] = self.modes
        t[:, 4:7] = re * self.amplitudes[:, None]
        t[:, 7:10] = im * self.amplitudes[:, None]
        return t, re, im

    def _pull_device_phases(self):
        """the device's phases (drive_device) back into the host state"""
        if getattr(self, "_dev_valid", False):
            self.phases = self._phases_dev.cpu().numpy().copy()
            self._dev_valid = False

    def drive_device(self, d, first, last, dt_dev):
        """GPU: the same update with dt read on the device (``dt_dev``, float64 [dt, ...] of the deferred time step,
        Propagator.defer_host): the host draws the step's normals (same engine, same order as update_noise: the RNG
        state and checkpoints are unchanged), one launch updates the phases in fp64 and writes the stirring table
        (csrc/hip/turbulence.hip turbPhasesKernel), then the stirring kernel. No host synchronization on dt."""
        dev = d.device
        if not getattr(self, "_dev_valid", False):
            self._phases_dev = torch.from_numpy(np.ascontiguousarray(self.phases, dtype=np.float64)).to(dev)
            self._kvec_dev = torch.from_numpy(np.ascontiguousarray(self.modes, dtype=np.float64)).to(dev)
            self._amps_dev = torch.from_numpy(np.ascontiguousarray(self.amplitudes, dtype=np.float64)).to(dev)
            self._table_dev = torch.empty(self.num_modes * 10, dtype=torch.float32, device=dev)
            self._dev_valid = True
        noise = torch.from_numpy(self.rng.normal(self.phases.size)).pin_memory()
        noise_dev = noise.to(dev, non_blocking=True)
        s = _lib.stream()
        _lib.hip().turbulence_phases(self.num_modes, self._phases_dev.data_ptr(), noise_dev.data_ptr(),
                                     self._kvec_dev.data_ptr(), self._amps_dev.data_ptr(), dt_dev.data_ptr(),
                                     self.decay_time, self.variance, self.sol_weight, self._table_dev.data_ptr(), s)
        self._dev_noise = noise  # (pinned source of the in-flight copy: kept until the next step)
        x, y, z, ax, ay, az = (d[f] for f in ("x", "y", "z", "ax", "ay", "az"))
        _lib.hip().compute_stirring(first, last, x.data_ptr(), y.data_ptr(), z.data_ptr(), ax.data_ptr(),
                                    ay.data_ptr(), az.data_ptr(), self.num_modes, self._table_dev.data_ptr(),
                                    self.sol_weight_norm, s)

    def drive(self, d, first, last, dt):
        self._pull_device_phases()
        self.update_noise(dt)
        table, re, im = self.mode_table()
        x, y, z, ax, ay, az = (d[f] for f in ("x", "y", "z", "ax", "ay", "az"))
        if d.device.type == "cuda":
            t = torch.from_numpy(table).to(d.device, non_blocking=True)
            self._dev_table = t  # keep alive until the kernel ran
            _lib.hip().compute_stirring(first, last, x.data_ptr(), y.data_ptr(), z.data_ptr(), ax.data_ptr(),
                                        ay.data_ptr(), az.data_ptr(), self.num_modes, t.data_ptr(),
                                        self.sol_weight_norm, _lib.stream())
        else:
            m = np.ascontiguousarray(self.modes)
            re, im, amp = np.ascontiguousarray(re), np.ascontiguousarray(im), np.ascontiguousarray(self.amplitudes)
            _lib.cpu().compute_stirring(first, last, x.data_ptr(), y.data_ptr(), z.data_ptr(), ax.data_ptr(),
                                        ay.data_ptr(), az.data_ptr(), self.num_modes, m.ctypes.data, re.ctypes.data,
                                        im.ctypes.data, amp.ctypes.data, self.sol_weight_norm)

    # ----------------------------------------------------------------------------------------- checkpointing
    def store(self, writer):
        self._pull_device_phases()
        p = self.PREFIX
        writer.step_attribute(p + "variance", self.variance)
        writer.step_attribute(p + "decayTime", self.decay_time)
        writer.step_attribute(p + "solWeight", self.sol_weight)
        writer.step_attribute(p + "solWeightNorm", self.sol_weight_norm)
        writer.step_attribute(p + "numModes", float(self.num_modes))
        writer.step_attribute(p + "modes", self.modes.reshape(-1))
        writer.step_attribute(p + "amplitudes", self.amplitudes)
        writer.step_attribute(p + "phases", self.phases)
        writer.step_attribute("rngEngineState", np.frombuffer(self.rng.state_text().encode(), dtype=np.int8))

    def load(self, attrs):
        p = self.PREFIX
        g = lambda k: np.asarray(attrs[p + k], dtype=np.float64).ravel()
        self.variance = float(g("variance")[0])
        self.decay_time = float(g("decayTime")[0])
        self.sol_weight = float(g("solWeight")[0])
        self.sol_weight_norm = float(g("solWeightNorm")[0])
        nm = int(g("numModes")[0])
        self.modes = g("modes").reshape(nm, 3)
        self.amplitudes = g("amplitudes")
        self.phases = g("phases")
        self._dev_valid = False  # (a device copy is re-made from these on the next device drive)
        if "rngEngineState" in attrs:
            raw = np.asarray(attrs["rngEngineState"]).ravel().astype(np.int8).tobytes()
            self.rng.set_state_text(raw.split(b"\0")[0].decode())


class TurbVeProp(HydroVeProp):
    # the stirring reads the new dt on the device when the host copy is deferred (TurbulenceData.drive_device), so
    # the step does not wait for it (Propagator.defer_host)
    needs_host_dt = False

    def __init__(self, out=sys.stdout, rank=0, av_clean=False, quiet=False, settings=None):
        super().__init__(out, rank, av_clean, quiet)
        self.turb = TurbulenceData(settings, rank == 0 and not quiet) if settings is not None else None

    def set_settings(self, settings):
        if self.turb is None:
            self.turb = TurbulenceData(settings, self.out is not None)

    def step(self, domain, d):
        self.compute_forces(domain, d)
        first, last = domain.start_index(), domain.end_index()
        self.compute_timestep(domain, d)
        self.timer.step("Timestep")
        dt_dev = getattr(d, "_dt_dev", None)
        if d.device.type == "cuda" and dt_dev is not None:
            self.turb.drive_device(d, first, last, dt_dev)
        else:
            self.turb.drive(d, first, last, d.minDt)
        self.timer.step("Turbulence Stirring")
        self.update_quantities(domain, d)
        self.timer.step("UpdateQuantities")
        self.timer.stop()

    def save(self, writer):
        self.turb.store(writer)

    def load(self, init_cond, reader):
        import os

        from ..utils.arg_parser import remove_modifiers
        from ..utils.io import H5PartReader

        path = remove_modifiers(init_cond)
        if not os.path.isfile(path):
            return
        step = init_cond.rsplit(":", 1)[1] if ":" in init_cond else "-1"
        rd = H5PartReader()
        rd.set_step(path, int(step) if step.lstrip("-").isdigit() else -1, collective=False)
        attrs = rd.step_attributes()
        rd.close_step()
        if self.turb is not None and TurbulenceData.PREFIX + "numModes" in attrs:
            self.turb.load(attrs)
            if self.out:
                print(f"Restored turbulence state from {path}:{step}", file=self.out)
