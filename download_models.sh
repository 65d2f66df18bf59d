#!/bin/bash
# Pretrained reference weights (raft-things/chairs/sintel/kitti/small .pth); they load as-is.
wget https://dl.dropboxusercontent.com/s/4j4z58wuv8o0mfz/models.zip
unzip models.zip
