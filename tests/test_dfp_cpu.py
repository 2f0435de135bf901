"""Digital-fingerprinting autoencoder (community/dfp; reference community/digital-human-security-analyst DFP
training stage): a per-user denoising autoencoder over mixed numeric / boolean / categorical log features, whose
reconstruction z-scores flag rows unlike the user's history."""
import numpy as np
import pandas as pd

from generativeaiexamples_amd.community.dfp import AEConfig, TabularAutoEncoder, train_per_user


def _logs(n, user, seed, anomalous=False):
    rng = np.random.default_rng(seed)
    hour = rng.normal(10 if user == "alice" else 20, 1.0, n)
    nbytes = rng.normal(5.0, 0.5, n)
    app = rng.choice(["mail", "wiki", "git"] if user == "alice" else ["crm", "mail"], n)
    vpn = rng.random(n) < 0.1
    if anomalous:
        hour, nbytes, app, vpn = rng.normal(3, 0.5, n), rng.normal(12.0, 0.5, n), np.array(["tor"] * n), np.ones(n, bool)
    return pd.DataFrame({"user": user, "hour": hour, "log_bytes": nbytes, "app": app, "vpn": vpn})


def test_autoencoder_scores_anomalies_above_normal_rows():
    train = _logs(2000, "alice", 0)
    feats = ["hour", "log_bytes", "app", "vpn"]
    ae = TabularAutoEncoder(AEConfig(encoder_layers=[64, 32], decoder_layers=[64], optimizer="adam",
                                     learning_rate=3e-3, batch_size=256), device="cpu")
    hist = ae.fit(train[feats], epochs=15)
    assert hist[-1] < hist[0]
    normal = ae.get_results(_logs(200, "alice", 1)[feats])
    odd = ae.get_results(_logs(50, "alice", 2, anomalous=True)[feats])
    assert {"hour_loss", "app_z_loss", "mean_abs_z", "max_abs_z"} <= set(normal.columns)
    assert odd["mean_abs_z"].min() > normal["mean_abs_z"].quantile(0.95)
    assert abs(normal["mean_abs_z"].mean()) < 2.0


def test_reference_defaults_and_per_user_models():
    cfg = AEConfig()
    assert (cfg.encoder_layers, cfg.decoder_layers, cfg.activation, cfg.swap_probability, cfg.learning_rate,
            cfg.learning_rate_decay, cfg.batch_size, cfg.optimizer) == ([512, 500], [512], "relu", 0.2, 1e-3, 0.99,
                                                                        512, "sgd")
    df = pd.concat([_logs(300, "alice", 3), _logs(300, "bob", 4)])
    models = train_per_user(df, "user", ["hour", "log_bytes", "app", "vpn"], epochs=2, device="cpu",
                            encoder_layers=[32], decoder_layers=[32])
    assert set(models) == {"alice", "bob"}
    # an unseen category maps to the "other" slot instead of failing
    r = models["bob"].get_results(_logs(5, "alice", 5)[["hour", "log_bytes", "app", "vpn"]])
    assert len(r) == 5 and np.isfinite(r["mean_abs_z"]).all()
