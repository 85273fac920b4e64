"""CPU tests of the orchestration layer: config registry (Appendix C), checkpoints (Appendix B),
schedulers, fault handling, trainer smoke runs of every family, entry-point CLIs."""
import math
import glob
import os
import subprocess
import sys

import pytest
import torch

from deep_vision_amd.config import CONFIGS, get_config, inception_poly
from deep_vision_amd.train import checkpoint as C
from deep_vision_amd.train.schedulers import LinearDecay, ManualPlateau, make_scheduler

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_appendix_c_configs():
    exp = {
        "lenet5": (64, "adam", {"lr": 1e-3}, "plateau", 50),
        "alexnet1": (128, "sgd", {"lr": 0.01, "momentum": 0.9, "weight_decay": 5e-4}, "plateau", 200),
        "alexnet2": (128, "sgd", {"lr": 0.01, "momentum": 0.9, "weight_decay": 5e-4}, "plateau", 200),
        "vgg16": (128, "sgd", {"lr": 0.01, "momentum": 0.9, "weight_decay": 5e-4}, "step", 200),
        "vgg19": (64, "sgd", {"lr": 0.01, "momentum": 0.9, "weight_decay": 5e-4}, "step", 200),
        "inception1": (128, "sgd", {"lr": 0.01, "momentum": 0.9, "weight_decay": 2e-4}, "lambda", 200),
        "resnet34": (256, "sgd", {"lr": 0.1, "momentum": 0.9, "weight_decay": 1e-4}, "plateau", 200),
        "resnet50": (256, "sgd", {"lr": 0.1, "momentum": 0.9, "weight_decay": 1e-4}, "plateau", 200),
        "mobilenet1": (128, "rmsprop", {"lr": 0.045, "alpha": 0.9, "eps": 1.0}, "step", 200),
        "yolov3": (16, "adam", {"lr": 0.01}, "manual_plateau", 300),
        "dcgan": (256, "adam", {"lr": 1e-4}, None, 50),
        "cyclegan": (4, "adam", {"lr": 2e-4, "betas": (0.5, 0.999)}, "linear_decay", 200),
    }
    for k, (bs, opt, op, sch, ep) in exp.items():
        c = CONFIGS[k]
        assert (c.batch_size, c.optimizer, c.optimizer_params, c.scheduler, c.total_epochs) == (bs, opt, op, sch, ep), k
    assert CONFIGS["vgg16"].scheduler_params == {"step_size": 10, "gamma": 0.5}
    assert CONFIGS["mobilenet1"].scheduler_params == {"step_size": 2, "gamma": 0.94}
    assert CONFIGS["yolov3"].batch_semantics == "per_replica" and CONFIGS["resnet50"].batch_semantics == "global"
    assert CONFIGS["resnet50"].per_rank_batch(8) == 32 and CONFIGS["yolov3"].global_batch(8) == 128
    assert inception_poly(0) == 1.0 and abs(inception_poly(15) - 0.75 ** 0.5) < 1e-12
    assert inception_poly(60) == 0.01 and inception_poly(80) == 0.001


def test_every_config_builds_its_model():
    from deep_vision_amd import models as M

    for name, c in CONFIGS.items():
        if c.family in ("dcgan", "cyclegan"):
            continue
        assert c.model in M.MODELS, name


def test_manual_plateau_counters():
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=1.0)
    s = ManualPlateau(opt, factor=0.1, max_patience=2)
    s.step()  # epoch 1
    assert s.patience_count == 1 and opt.param_groups[0]["lr"] == 1.0
    s.update(5.0)
    s.step()  # new best -> counter resets to 0 then increments
    assert s.patience_count == 1
    for v in (6.0, 7.0, 8.0):
        s.update(v)
        s.step()
    # counts 2, 3 -> > 2 triggers the decay on the next call
    assert opt.param_groups[0]["lr"] == pytest.approx(0.1)
    h = ManualPlateau(opt, max_patience=2, inclusive=True)
    h.update(1.0)
    for _ in range(2):
        h.update(2.0)
        h.step()
    h.step()
    assert h.current_learning_rate == pytest.approx(0.01)


def test_linear_decay():
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=2e-4)
    s = LinearDecay(opt, 2e-4, total_steps=200, step_decay=100)
    for _ in range(150):
        s.step()
    assert opt.param_groups[0]["lr"] == pytest.approx(1e-4)
    st = s.state_dict()
    s2 = LinearDecay(opt, 2e-4, 200, 100)
    s2.load_state_dict(st)
    assert s2.current_learning_rate == pytest.approx(1e-4)


def test_checkpoint_names_and_module_prefix(tmp_path):
    assert C.classifier_checkpoint_name("resnet50", "2019-01-03T10:00:00", 7) == "resnet50-2019-01-03T10:00:00-epoch-7.pt"
    assert C.best_model_name("1.0.1", 56, 42.01434) == "model-v1.0.1-epoch-56-loss-42.0143.pt"
    assert C.epoch_from_name("./models/model-v1.0.1-epoch-56-loss-42.0143.pt") == 56
    m = torch.nn.Linear(3, 2)
    sd = {"module." + k: v for k, v in m.state_dict().items()}
    path = str(tmp_path / "x-epoch-3.pt")
    C.atomic_save({"epoch": 3, "model": sd, "optimizer": None, "scheduler": None, "loggers": C.initialize_loggers()},
                  path)
    m2 = torch.nn.Linear(3, 2)
    _, _, _, loggers, start = C.load_checkpoint(path, m2)
    assert start == 4 and set(loggers) == set(C.LOGGER_KEYS)
    assert torch.equal(m2.weight, m.weight)
    mgr = C.CheckpointManager(str(tmp_path / "ck"), max_to_keep=2)
    for i in range(4):
        mgr.save({"step": i})
    assert sorted(os.listdir(tmp_path / "ck")) == ["ckpt-3.pt", "ckpt-4.pt"]
    assert C.latest(str(tmp_path / "ck")).endswith("ckpt-4.pt")


def test_classifier_resume_continues(tmp_path):
    from deep_vision_amd.train.classification import run_epochs

    cfg = get_config("lenet5")
    kw = dict(device="cpu", synthetic=True, synthetic_size=128, num_workers=0, checkpoint_dir=str(tmp_path) + "/",
              max_steps=4, val_steps=1)
    last, loggers = run_epochs(cfg, None, epochs=2, **kw)
    ck = C.load(last)
    assert list(ck)[:5] == ["epoch", "model", "optimizer", "scheduler", "loggers"] and ck["epoch"] == 2
    assert len(ck["loggers"]["val_top1_acc"]["value"]) == 3  # epoch 0 + 2 epochs
    last2, loggers2 = run_epochs(cfg, last, epochs=3, **kw)
    ck2 = C.load(last2)
    assert ck2["epoch"] == 3 and len(ck2["loggers"]["val_top1_acc"]["value"]) == 5  # resumed loggers + val(0) + e3


def test_fault_injection_and_nonfinite_skip(monkeypatch):
    from deep_vision_amd.train.engine import Engine
    from deep_vision_amd.train.optim import FusedSGD

    monkeypatch.setenv("DV_FAULT", "nan_loss@2")
    monkeypatch.setenv("DV_NAN_CHECK", "step")
    eng = Engine(device="cpu")
    m = torch.nn.Linear(4, 1)
    opt = FusedSGD(m.parameters(), lr=0.1)
    x = torch.randn(8, 4)
    w0 = m.weight.detach().clone()
    assert eng.backward_step(m(x).pow(2).mean(), m, opt)
    w1 = m.weight.detach().clone()
    assert not torch.equal(w0, w1)
    assert not eng.backward_step(m(x).pow(2).mean(), m, opt)  # injected NaN: skipped
    assert torch.equal(m.weight.detach(), w1) and eng.guard.skipped == 1
    assert eng.backward_step(m(x).pow(2).mean(), m, opt)


@pytest.mark.parametrize("name,size,extra", [("yolov3", 64, {}), ("hourglass", 64, {"num_stack": 2}),
                                             ("centernet", 128, {"num_classes": 4})])
def test_family_trainers_smoke(tmp_path, name, size, extra):
    from deep_vision_amd.train.detection import train

    cfg = get_config(name, input_shape=(3, size, size), batch_size=2)
    cfg = cfg.replace(model_params={**cfg.model_params, **extra})
    best = train(cfg, synthetic=True, synthetic_size=4, epochs=1, device="cpu", workers=0, log_every=1,
                 checkpoint_dir=str(tmp_path), tensorboard_dir=str(tmp_path / "tb"))
    assert best and os.path.basename(best).startswith("model-v") and C.epoch_from_name(best) == 1
    # TensorBoard streams with the reference tags (YOLO/CenterNet: train + val writers)
    from deep_vision_amd.utils.tensorboard import read_scalars

    tags = {}
    for f in glob.glob(str(tmp_path / "tb" / "**" / "events.out.tfevents.*"), recursive=True):
        tags.update(read_scalars(f))
    assert {"epoch train loss", "epoch val loss"} <= set(tags)
    if name == "yolov3":
        assert {"batch train loss", "batch xy loss", "batch class loss"} <= set(tags)
    if name == "hourglass":
        assert "epoch learning rate" in tags


def test_gan_trainers_smoke(tmp_path):
    from deep_vision_amd.train.gan import ImagePool, train_cyclegan, train_dcgan

    assert train_dcgan(epochs=2, batch_size=8, synthetic=True, synthetic_size=16, device="cpu",
                       checkpoint_dir=str(tmp_path / "dc"), max_steps=2).endswith("ckpt-1.pt")
    assert train_cyclegan("toy", 1, 2, True, synthetic_size=1, size=32, n_blocks=1, device="cpu",
                          checkpoint_dir=str(tmp_path / "cg-{dataset}"),
                          tensorboard_dir=str(tmp_path / "tb")).endswith("ckpt-1.pt")
    from deep_vision_amd.utils.tensorboard import read_scalars

    ev = glob.glob(str(tmp_path / "tb" / "toy" / "*" / "train" / "events.out.tfevents.*"))
    sc = read_scalars(ev[0])
    assert len(sc) == 12 and [s for s, _, _ in sc["loss_gen_total"]] == [1, 2]
    pool = ImagePool(2)
    a = torch.randn(3, 1, 2, 2)
    out = pool.query(a)
    assert torch.equal(out[:2], a[:2]) and pool.count == 2


def test_entry_point_cli(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "LeNet/pytorch/train.py"), "-m", "lenet5", "--synthetic",
                        "--epochs", "1", "--max-steps", "2", "--val-steps", "1", "--workers", "0", "--device", "cpu",
                        "--checkpoint-dir", str(tmp_path) + "/"], capture_output=True, text=True, cwd=str(tmp_path),
                       env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Validation Top 1 acc" in r.stdout and any(f.startswith("lenet5-") for f in os.listdir(tmp_path))


@pytest.mark.parametrize("fam,target,model", [("ResNet/pytorch", "train_resnet50", "resnet50"),
                                              ("ResNet/tensorflow", "train_resnet152", "resnet152"),
                                              ("AlexNet/tensorflow", "train_alexnet2", "alexnet2"),
                                              ("LeNet/tensorflow", "train_lenet5", "lenet5")])
def test_family_makefile_targets(fam, target, model):
    """The reference's run UX (R/<Family>/<fw>/Makefile): `make train_<model>` starts a nohup'ed
    train.py -m <model> writing <model>-<time>.log (dry run: the command line only)."""
    import os
    import shutil
    import subprocess

    if shutil.which("make") is None:
        pytest.skip("make not installed")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run(["make", "-n", "-C", os.path.join(root, fam), target], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert f"train.py -m {model}" in r.stdout and "nohup" in r.stdout and f"{model}-" in r.stdout
