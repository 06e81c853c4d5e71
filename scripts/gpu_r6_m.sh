#!/bin/bash
# Round 6: SQ PMC (bank conflicts, issue) of the narrow 3x3 weight gradient at 18 / 36
# channels with the padded halo rows (new) and the unpadded ones (base)
cd "$GRAFT_REPO_ROOT" || exit 1
for lib in new base; do
  if [ $lib = new ]; then L=vae-2_amd/vae2/libvae2_hip.so; else L=vae-2_amd/vae2/libvae2_hip_base.so; fi
  for only in 3 4; do
    VAE2_LIB=$PWD/$L bash scripts/gpu_sqpmc.sh r6_m_${lib}_$only $only wgrad3n_kernel || exit 1
  done
done
