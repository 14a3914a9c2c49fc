"""MI355X-native FIA (fast influence analysis) for latent factor models.

Drop-in for the reference's influence path (zz9tf/FIA-KDD-19 src/influence):
    from influence.matrix_factorization import MF
    from influence.NCF import NCF
    model.get_influence_on_test_loss([test_idx], np.arange(n_train))
All compute runs in libfia.so (HIP, gfx950); see include/fia.h.
"""
