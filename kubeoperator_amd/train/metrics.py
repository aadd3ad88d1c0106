"""Prometheus metrics of a training run (tokens/s, step time, loss, grad norm, collective
time), served by rank 0 on ``--metrics-port`` so the cluster's Prometheus (the ``cluster-addon`` role's
scrape config picks up ``prometheus.io/scrape`` pod annotations) records the job beside the AMD GPU
exporter's device metrics.
"""
from __future__ import annotations


class TrainMetrics:
    def __init__(self, port: int, labels: dict):
        from prometheus_client import CollectorRegistry, Counter, Gauge, start_http_server

        self.registry = CollectorRegistry()
        names = sorted(labels)
        self.labels = [labels[n] for n in names]

        def gauge(name, doc):
            return Gauge(name, doc, names, registry=self.registry).labels(*self.labels)

        self.step = gauge("kop_train_step", "optimizer steps completed")
        self.loss = gauge("kop_train_loss", "mean training loss of the last logged step")
        self.grad_norm = gauge("kop_train_grad_norm", "global gradient norm before clipping")
        self.lr = gauge("kop_train_learning_rate", "learning rate of the last step")
        self.step_seconds = gauge("kop_train_step_seconds", "wall time of the last logged step (max over ranks)")
        self.tokens_per_s = gauge("kop_train_tokens_per_second", "whole-job training throughput")
        self.tflops = gauge("kop_train_tflops_per_gpu", "model FLOP/s per GPU (6N + attention)")
        self.comm_bytes = Counter("kop_train_collective_bytes", "gradient bytes handed to RCCL collectives",
                                  names, registry=self.registry).labels(*self.labels)
        self.server = start_http_server(port, registry=self.registry)

    def observe(self, *, step, loss, grad_norm, lr, step_s, tokens_per_s, tflops, comm_bytes_delta=0):
        self.step.set(step)
        self.loss.set(loss)
        self.grad_norm.set(grad_norm)
        self.lr.set(lr)
        self.step_seconds.set(step_s)
        self.tokens_per_s.set(tokens_per_s)
        self.tflops.set(tflops)
        if comm_bytes_delta:
            self.comm_bytes.inc(comm_bytes_delta)

    def close(self):
        srv = self.server[0] if isinstance(self.server, tuple) else None
        if srv is not None:
            srv.shutdown()
