"""vae2 — MI355X-native VAE² ELBO training path (HIP kernels via libvae2_hip.so).

Public surface mirrors the reference's:
  vae2.hrnet      get_encdec_model / get_encz_model / get_D_*_model
  vae2.model      FullModel_encdec
  vae2.criterion  L1Loss / KLLoss / lsgan_adversarial_loss
  vae2.optim      FusedAdam (torch.optim.Adam semantics over flat buffers)
  vae2.dist       RCCL data parallelism + SyncBN statistics
  vae2.config     yacs-compatible CfgNode
"""
__version__ = "0.1.0"
