"""Output formats of the Algorithm-1 driver (hybrid_NF_MCMC/main_algorithm_1.py),
written from the batched engine's device results:

  sample tuples            MonteCarlo.sample (MCMC/monte_carlo.py:416-444)
  sampled_data.csv         main_algorithm_1.py:499-534 (one row per sample() tuple)
  mc_run_configs.npy       main_algorithm_1.py:537-541 (stacked sample configurations)
  mc_run_testing_configs.npy  main_algorithm_1.py:544-547
  params.json              main_algorithm_1.py:131-134 (json, indent 4)
  acceptance_rate_data.csv main_algorithm_1.py:434-440
  model .pth               torch.save(model.state_dict()) (main_algorithm_1.py:327)

The batched engine returns sample() snapshots as device arrays (E, W and the
configuration at each sampled step); `sample_tuples` turns one chain's snapshots
into the reference's tuples with the reference's arithmetic.
"""
import csv
import json
import os

import numpy as np


def sample_tuple(cycle_number, total_energy, total_virial, num_particles, box_x, box_y, beta, particles):
    """(cycle, E/N, rho, P, box_x, box_y, particles) as monte_carlo.py:420-444 computes it."""
    volume = box_x * box_y  # SimulationBox.volume (simulation_box.py:17)
    energy_per_particle = total_energy / num_particles
    density = num_particles / volume
    pressure = density / beta + total_virial / (2.0 * volume)
    return (cycle_number, energy_per_particle, density, pressure, box_x, box_y, np.array(particles, copy=True))


def sample_tuples(bmc, samples_xy, samples_ew, chain, step0, sample_every, n_moves):
    """One chain's sample() tuples from BatchedMonteCarlo.local_moves(..., sample_every)
    outputs; particles come back in the chain's reference dtype."""
    steps = [s for s in range(step0 + 1, step0 + n_moves + 1) if s % sample_every == 0]
    xy = samples_xy[chain].cpu().numpy()
    ew = samples_ew[chain].cpu().numpy()
    f32 = bool(bmc.state_is_f32[chain].item())
    out = []
    for k, s in enumerate(steps):
        p = xy[k].astype(np.float32) if f32 else xy[k]
        out.append(sample_tuple(s, np.float64(ew[k, 0]), np.float64(ew[k, 1]), bmc.N, np.float64(bmc.phys.box_x),
                                np.float64(bmc.phys.box_y), bmc.phys.beta, p))
    return out


def write_sampled_data(path, local_samples):
    """sampled_data.csv of one run (main_algorithm_1.py:499-534)."""
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["cycle_number", "energy_per_particle", "density", "pressure", "box_size_x", "box_size_y",
                    "particle_configuration"])
        for cycle, epp, rho, p, bx, by, particles in local_samples:
            w.writerow([cycle, epp, rho, p, bx, by, np.array(particles).flatten().tolist()])


def save_configs(path, samples):
    """mc_run_configs.npy / mc_run_testing_configs.npy: np.array of the configurations
    (sample[6] of each tuple, or the configurations themselves)."""
    cfgs = [s[6] if isinstance(s, tuple) else s for s in samples]
    np.save(path, np.array(cfgs))


def write_params(path, params):
    with open(path, "w") as f:
        json.dump(params, f, indent=4)


def write_acceptance_rate(path, steps_history, p_acc_history):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["MCMC_Steps", "Acceptance_Rate"])
        for s, a in zip(steps_history, p_acc_history):
            w.writerow([s, a])


def write_run_dir(run_dir, local_samples, testing_samples=None):
    """The per-run files of main_algorithm_1.py:499-547."""
    os.makedirs(run_dir, exist_ok=True)
    write_sampled_data(os.path.join(run_dir, "sampled_data.csv"), local_samples)
    save_configs(os.path.join(run_dir, "mc_run_configs.npy"), local_samples)
    save_configs(os.path.join(run_dir, "mc_run_testing_configs.npy"), testing_samples or [])
