"""BiLSTM + attention-pooling speech model (`pytorch_model.py:156-242`).

The reference version cannot run (F9): it calls ``pad_packed_sequence`` on a
plain tensor, builds its mask with a hard-coded ``.cuda()`` and feeds the
packed output of layer 1 into layer 2.  This is the repaired model: same
parameter tree (``lstm1``, ``atten1``, ``lstm2``, ``atten2``, ``fc1``, ``fc2``),
optional per-sample ``lengths`` (defaults to full length), a device-agnostic
mask, and layer 2 consuming layer 1's padded output.  The LSTM cells run on
PyTorch-ROCm (MIOpen RNN); SURVEY K13 scopes a hand-written RNN kernel out.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F


class Attention(nn.Module):
    def __init__(self, hidden_size, batch_first=False):
        super().__init__()
        self.hidden_size = hidden_size
        self.batch_first = batch_first
        self.att_weights = nn.Parameter(torch.empty(1, hidden_size))
        stdv = 1.0 / math.sqrt(hidden_size)
        nn.init.uniform_(self.att_weights, -stdv, stdv)

    def forward(self, inputs, lengths=None):
        if not self.batch_first:
            inputs = inputs.transpose(0, 1)
        batch_size, max_len = inputs.shape[:2]
        weights = torch.matmul(inputs, self.att_weights.t()).squeeze(-1)   # [B, T]
        attentions = torch.softmax(F.relu(weights), dim=-1)
        if lengths is not None:
            lengths = torch.as_tensor(lengths, device=inputs.device)
            mask = (torch.arange(max_len, device=inputs.device)[None, :] < lengths[:, None])
            attentions = attentions * mask.to(attentions.dtype)
            attentions = attentions / attentions.sum(-1, keepdim=True).clamp_min(1e-12)
        representations = (inputs * attentions.unsqueeze(-1)).sum(1)
        return representations, attentions


class MyLSTM(nn.Module):
    def __init__(self, feature_dim, num_classes, hidden_dim=512, lstm_layer=2, dropout=0.2):
        super().__init__()
        self.dropout = nn.Dropout(p=dropout)
        self.lstm1 = nn.LSTM(feature_dim, hidden_dim, num_layers=1, bidirectional=True)
        self.atten1 = Attention(hidden_dim * 2, batch_first=True)
        self.lstm2 = nn.LSTM(hidden_dim * 2, hidden_dim, num_layers=1, bidirectional=True)
        self.atten2 = Attention(hidden_dim * 2, batch_first=True)
        width = hidden_dim * lstm_layer * 2
        self.fc1 = nn.Sequential(nn.Linear(width, width), nn.BatchNorm1d(width), nn.ReLU())
        self.fc2 = nn.Linear(width, num_classes)

    def forward(self, x, lengths=None):
        # x: [B, 1, F, T] spectrogram (or [B, F, T]) -> time-major [T, B, F]
        if x.dim() == 4:
            x = x.squeeze(1)
        x = x.permute(2, 0, 1)
        out1, _ = self.lstm1(x)
        a, _ = self.atten1(out1.transpose(0, 1), lengths)
        out2, _ = self.lstm2(out1)
        b, _ = self.atten2(out2.transpose(0, 1), lengths)
        z = torch.cat([a, b], dim=1)
        z = self.fc1(self.dropout(z))
        return self.fc2(self.dropout(z))
