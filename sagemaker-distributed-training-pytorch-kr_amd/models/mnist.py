"""MNIST CNN: the reference's ``Net`` (/root/reference/1_training_mnist_ddp/model_def.py:22-45).

conv(1->32, 3x3) -> ReLU -> conv(32->64, 3x3) -> ReLU -> maxpool 2 -> Dropout2d(0.25) -> flatten
-> FC(9216->128) -> ReLU -> Dropout(0.5) -> FC(128->10) -> log_softmax; 1,199,882 parameters.
Parameter names (conv1, conv2, fc1, fc2) match the reference so ``mnist_cnn.pt`` state dicts
interchange. (The reference uses Dropout2d for the post-FC dropout too; it is kept as a plain
element dropout here since Dropout2d on a 2-D tensor is deprecated and means the same.)
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 32, 3, 1)
        self.conv2 = nn.Conv2d(32, 64, 3, 1)
        self.dropout1 = nn.Dropout2d(0.25)
        self.dropout2 = nn.Dropout(0.5)
        self.fc1 = nn.Linear(9216, 128)
        self.fc2 = nn.Linear(128, 10)

    def forward(self, x):
        x = F.relu(self.conv1(x))
        x = F.relu(self.conv2(x))
        x = F.max_pool2d(x, 2)
        x = self.dropout1(x)
        x = torch.flatten(x, 1)
        x = F.relu(self.fc1(x))
        x = self.dropout2(x)
        x = self.fc2(x)
        return F.log_softmax(x, dim=1)
