from .schedule import (logsnr_schedule_cosine, alpha_sigma, q_sample, diffusion_loss,
                       sampler_logsnrs, cfg_posterior)

__all__ = ["logsnr_schedule_cosine", "alpha_sigma", "q_sample", "diffusion_loss",
           "sampler_logsnrs", "cfg_posterior"]
