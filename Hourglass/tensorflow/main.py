"""Stacked Hourglass click CLI (R/Hourglass/tensorflow/main.py:21-66).

Same options and defaults (including ``--num_heatmap 442``); the GCS upload of the
best model becomes a copy into ``<output_bucket>/<output_dir>/`` on the local filesystem (no
network here), and its path is written to ``/tmp/output.txt`` like the reference.

Like the reference container's ``python3 main.py`` under MirroredStrategy
(R/Hourglass/tensorflow/train.py:195, Dockerfile:19) it trains on every visible GPU by default:
one process per GPU (``--nproc``, default all visible, counted without initialising HIP), the
whole step captured and replayed as a HIP graph (``--graph`` default; ``--no-graph`` for eager).
"""
import os
import shutil
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

import click  # noqa: E402

from deep_vision_amd.config import get_config  # noqa: E402
from deep_vision_amd.train.detection import train  # noqa: E402


@click.command()
@click.option("--epochs", default=100, help="Total number of epochs.")
@click.option("--start_epoch", default=1, help="The initial epoch to start with.")
@click.option("--learning_rate", default=0.001, help="The learning rate to start with.")
@click.option("--tensorboard_dir", default="./logs", help="The directory to store Tensorboard events.")
@click.option("--checkpoint", help="The path to checkpoint file.")
@click.option("--num_heatmap", default=442, help="Number of heatmap layers.")
@click.option("--batch_size", default=32, help="Size of a mini batch.")
@click.option("--train_tfrecords", help="Location of training TF Records.")
@click.option("--val_tfrecords", help="Location of validation TF Records.")
@click.option("--output_bucket", help="Output location (local directory here).")
@click.option("--output_dir", help="Directory name under the output location.")
@click.option("--version", default="0.0.1", help="Version number of the new model.")
@click.option("--synthetic", is_flag=True, help="Synthetic data (no TFRecords needed).")
@click.option("--device", default=None)
@click.option("--nproc", type=int, default=None, help="Processes, one per GPU (default: every visible GPU).")
@click.option("--graph/--no-graph", default=None,
              help="HIP-graph replay of the training step (default: on, Hourglass's measured-faster mode).")
@click.option("--max_steps", type=int, default=None, help="Stop after this many training steps (smoke runs).")
@click.option("--input_size", type=int, default=None, help="Square input size (default 256).")
@click.option("--num_stack", type=int, default=None, help="Hourglass stacks (default 4).")
def main(epochs, start_epoch, learning_rate, tensorboard_dir, checkpoint, num_heatmap, batch_size, train_tfrecords,
         val_tfrecords, output_bucket, output_dir, version, synthetic, device, nproc, graph, max_steps, input_size,
         num_stack):
    from deep_vision_amd.launch import maybe_spawn

    graph = maybe_spawn(nproc, device, graph=graph, model="hourglass")  # parent: spawns one rank per GPU and exits; ranks: CPU pinning
    cfg = get_config("hourglass")
    cfg = cfg.replace(optimizer_params={"lr": learning_rate}, batch_size=batch_size, total_epochs=epochs,
                      model_params={**cfg.model_params, "num_heatmap": num_heatmap},
                      extras={**cfg.extras, "version": version})
    if input_size:
        cfg = cfg.replace(input_shape=(3, input_size, input_size))
    if num_stack:
        cfg = cfg.replace(model_params={**cfg.model_params, "num_stack": num_stack})
    model_path = train(cfg, checkpoint, train_glob=train_tfrecords, val_glob=val_tfrecords, synthetic=synthetic,
                       device=device, tensorboard_dir=tensorboard_dir, graph=graph, max_steps=max_steps)
    print("Received model " + str(model_path))
    if output_bucket is None or output_dir is None or model_path is None:
        return
    dst_dir = os.path.join(output_bucket, output_dir)
    os.makedirs(dst_dir, exist_ok=True)
    out = shutil.copy(model_path, dst_dir)
    print("Copied model file to " + out)
    with open("/tmp/output.txt", "w") as fp:
        fp.write(out + "\n")
        print("Saved output to /tmp/output.txt")


if __name__ == "__main__":
    main()
